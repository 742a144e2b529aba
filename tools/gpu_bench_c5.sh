set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --steps 10 --warmup 2 --c5-steps 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_c5.err; exit 11; }
cat gpurun_out/bench_c5.json
