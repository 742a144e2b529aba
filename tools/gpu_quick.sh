# Quick batched-kernel check: GPU parity tests of the batched path, phase stamps, C3 bench.
# usage: gpurun -- 'bash tools/gpu_quick.sh TAG'
set -o pipefail
TAG=${1:-quick}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_batched_gpu.py tests/test_algos_gpu.py tests/test_oracle_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 100 python tools/stamps_batched.py > $O/stamps.log 2>&1 || { echo "stamps rc=$?"; tail -5 $O/stamps.log; exit 2; }
grep PCX_STAMPS $O/stamps.log | tail -1
timeout -k 10 100 python bench.py --no-cpu-baseline --c5-steps 0 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('C3 %.2fM rounds/s kernel %.3f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))"
