# rocprofv3 evidence for the bench kernels: kernel-trace stats of the default bench
# command, then one FETCH_SIZE, one WRITE_SIZE and one SQ_INSTS_VALU counter pass (separate runs, as
# MI355X_MICROARCH.md prescribes), summarised into gpurun_out/$TAG/pmc_traffic.json.
# usage: gpurun --timeout 900 -- 'bash tools/gpu_profile.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --c5-steps 1 --no-c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS > $O/kt.log 2>&1 || { echo "kernel-trace rc=$?"; tail -5 $O/kt.log; exit 12; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 bench.py $ARGS > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $O/fetch.log; exit 13; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 bench.py $ARGS > $O/write.log 2>&1 || { echo "write rc=$?"; tail -5 $O/write.log; exit 14; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $O/valu -o pmc -- python3 bench.py $ARGS > $O/valu.log 2>&1 || { echo "valu rc=$?"; tail -5 $O/valu.log; exit 16; }
KS=$(find $O/kt -name "kt_kernel_stats.csv" | head -1)
FC=$(find $O/fetch -name "pmc_counter_collection.csv" | head -1)
WC=$(find $O/write -name "pmc_counter_collection.csv" | head -1)
VC=$(find $O/valu -name "pmc_counter_collection.csv" | head -1)
python3 tools/pmc_summary.py --stats "$KS" --fetch "$FC" --write "$WC" --valu "$VC" --out $O/pmc_traffic.json \
    --note "bench.py $ARGS (C3 65536 x 50x20 with every output + one C5 1M x 4k), MI355X" > $O/summary.log 2>&1 || { echo summary failed; tail -5 $O/summary.log; exit 15; }
cp "$KS" $O/kernel_stats.csv
echo profile ok
