# Kernel trace (rocprofv3 --kernel-trace --stats) of one C5 consensus (plus warmup).
# usage: gpurun -- 'bash tools/gpu_c5_ktrace.sh TAG'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-c5kt}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c4 --c5-steps 1 > $O/kt.log 2>&1 || { echo "rc=$?"; tail -5 $O/kt.log; exit 1; }
KS=$(find $O/kt -name "kt_kernel_stats.csv" | head -1)
cp "$KS" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
    print("%-60s calls %5s  avg %10.3f ms  total %10.3f ms" % (n, r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
