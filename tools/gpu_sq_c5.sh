# SQ counters of the C5 matrix-pipeline kernels (one consensus), pass 1 of gpu_sq_counters.sh's set:
# how busy the VALU / LDS pipes are in the column passes and the selection histogram.
# usage: gpurun -- 'bash tools/gpu_sq_c5.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sqc5}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 1 --warmup 0 --rounds 4096 --no-cpu-baseline --c5-steps 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- python3 bench.py $ARGS > $O/p1.log 2>&1 || { echo "pass1 rc=$?"; tail -5 $O/p1.log; exit 1; }
python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
O = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in ("k_colstats", "k_wcd", "k_outcomes", "k_gemv2", "k_scores_wcd", "k_sel_hist", "k_sel_init", "k_syrk"):
            if k + "(" in n:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    med = {c: sorted(v)[len(v) // 2] for c, v in vals[k].items()}
    # VALU issue time if every wave64 VALU instruction holds its SIMD 4 cycles (16 lanes a
    # cycle, fp64 included on gfx950), spread over 1024 SIMDs at 2.4 GHz; compare with the
    # kernel's duration to see how close to VALU-issue bound it is
    line = " ".join("%s=%.4g" % (c, v) for c, v in sorted(med.items()))
    extra = "  valu_issue_ms_est=%.2f" % (med.get("SQ_INSTS_VALU", 0) * 4 / 1024 / 2.4e9 * 1e3)
    print(k, line + extra)
PY
