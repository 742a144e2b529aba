# Round-3 profiling pass: the C3 kernel's phase stamps, one C5 shard's stage times, a short bench.
# usage: gpurun --timeout 900 -- 'bash tools/gpu_prof_r3.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_boundary_gpu.py -q -k survives --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 11; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u tools/stamps_batched.py > $O/stamps.log 2>&1 || { echo "stamps rc=$?"; tail -20 $O/stamps.log; exit 12; }
grep PCX_STAMPS $O/stamps.log | tail -2
timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 13; }
cat $O/w8.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c4 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 14; }
python -c "import json,sys; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'], d['c5']['latency_ms'], d['c5']['stage_ms'])"
