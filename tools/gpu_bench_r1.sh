set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r1.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_r1 -o pmc -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_r1.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_r1 -o pmc -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_r1.log 2>&1 || exit 14
cat gpurun_out/bench_r1.json
find gpurun_out -name "*.csv" | head -20
