# Single-matrix path check after a pipeline change: its GPU tests, then one C5 shard's stage
# times and the 1-GPU C5 latency.  usage: gpurun --timeout 1200 -- 'bash tools/gpu_matrix_check.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-mcheck}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_matrix_gpu.py tests/test_c5_gpu.py tests/test_boundary_gpu.py tests/test_dist_gpu.py tests/test_algos_gpu.py tests/test_cov_grid_gpu.py tests/test_oracle_gpu.py -q -x --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 11; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 13; }
cat $O/w8.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c4 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 14; }
python -c "import json,sys; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'], d['c5']['latency_ms'], d['c5']['stage_ms'])"
