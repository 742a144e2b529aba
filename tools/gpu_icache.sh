# Instruction-cache and issue-stall counters of the C3 batched launch (one --pmc pass each),
# for the libpcx builds given (PCX_LIB).  usage: gpurun -- 'bash tools/gpu_icache.sh TAG LIB...'
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -oE "SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_WAIT_INST_ANY|SQ_INSTS_VALU\b" $O/counters.txt | sort -u | head -20
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --c5-steps 0 --no-c4"
have() { grep -q -w "$1" $O/counters.txt; }
P1=""; for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do have $c && P1="$P1 $c"; done
P2=""; for c in SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU; do have $c && P2="$P2 $c"; done
echo "pass1:$P1"; echo "pass2:$P2"
for L in "$@"; do
  N=$(basename $(dirname $L))
  for k in 1 2; do
    C=$P1; [ $k = 2 ] && C=$P2
    [ -z "$C" ] && continue
    PCX_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/$N$k -o pmc -- python3 bench.py $ARGS > $O/$N$k.log 2>&1 || { echo "pmc rc=$? ($N pass $k)"; tail -5 $O/$N$k.log; exit 1; }
  done
  python3 - "$O/$N" "$N" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "batched_round_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], " ".join("%s=%.4g" % (k, sorted(v)[len(v) // 2]) for k, v in sorted(vals.items())))
PY
done
