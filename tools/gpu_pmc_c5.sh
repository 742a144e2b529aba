# PMC passes over one C5 consensus (1M x 4096, 1 GPU): SQ issue / MFMA / VALU, HBM FETCH and
# WRITE, L2 hit/miss, LDS -- one rocprofv3 --pmc run per pass, summarised per kernel (median).
# usage: gpurun -- 'bash tools/gpu_pmc_c5.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-pmcc5}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 1 --warmup 0 --rounds 4096 --no-cpu-baseline --no-c4 --c5-steps 1"
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
         "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o pmc -- python3 bench.py $ARGS > $O/p$i.log 2>&1 || { echo "pass$i rc=$?"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections, re
O = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
seen = {}
for f in glob.glob(O + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "pcx::" not in n:
            continue
        m = re.search(r"(k_[a-z0-9_]+)", n)
        k = m.group(1) if m else n[:40]
        if "k_gemm_i8" in k:  # launches alternate: grid x grid, then the mixed block
            key = (f, r["Counter_Name"])
            seen[key] = seen.get(key, -1) + 1
            k += "_grid" if seen[key] % 2 == 0 else "_mixed"
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    med = {c: sorted(v)[len(v) // 2] for c, v in vals[k].items()}
    if med.get("SQ_WAVE_CYCLES", 0) == 0 and med.get("FETCH_SIZE", 0) < 1e5:
        continue
    gb = (2 * med.get("FETCH_SIZE", 0) * 1024 + med.get("WRITE_SIZE", 0) * 1024) / 1e9
    print("%-22s hbm_GB=%.2f " % (k, gb) + " ".join("%s=%.4g" % (c, v) for c, v in sorted(med.items())))
PY
