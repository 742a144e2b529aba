# SQ counters of the C3 batched launch (two --pmc passes, each within the 8 SQ / 2 GRBM slots).
# usage: gpurun -- 'bash tools/gpu_sq_counters.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sq}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --c5-steps 0 --no-c4"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- python3 bench.py $ARGS > $O/p1.log 2>&1 || { echo "pass1 rc=$?"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC --output-format csv -d $O/p2 -o pmc -- python3 bench.py $ARGS > $O/p2.log 2>&1 || { echo "pass2 rc=$?"; tail -5 $O/p2.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(O + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "batched_round_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = sorted(vals[k]); print("%-24s median %.4g  (n=%d)" % (k, v[len(v) // 2], len(v)))
PY
