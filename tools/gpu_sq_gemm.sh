# SQ counters of the int8 covariance GEMM (k_gemm_i8) in one C5 consensus: where its
# waves spend their cycles (MFMA busy, waits, LDS).  usage: gpurun -- 'bash tools/gpu_sq_gemm.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sqgemm}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 1 --warmup 0 --rounds 4096 --no-cpu-baseline --no-c4 --c5-steps 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- python3 bench.py $ARGS > $O/p1.log 2>&1 || { echo "pass1 rc=$?"; tail -5 $O/p1.log; exit 1; }
python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
O = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in ("k_gemm_i8", "k_syrk", "k_digits", "k_wcd"):
            if k + "(" in n:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    print(k, " ".join("%s=%s" % (c, [round(x) for x in v]) for c, v in sorted(vals[k].items())))
PY
