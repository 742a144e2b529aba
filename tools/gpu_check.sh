# One GPU call: GPU parity tests, smoke, bench (C3 + C5), rocprofv3 kernel stats of the bench.
# usage (from the build container): gpurun --timeout 1100 -- 'bash tools/gpu_check.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 11; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 12; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 13; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c5-steps 2 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 14; }
find $O/prof -name "*stats*.csv" | head
