# Kernel trace of the bench's C4 entry (100k x 1k, integer reputations): per-launch times of the
# power iteration, the hard replay and the selection.   gpurun -- 'bash tools/kt_c4.sh TAG'
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c5-steps 0 > $O/kt_c4.log 2>&1 || { echo "kt rc=$?"; tail -5 $O/kt_c4.log; exit 1; }
echo ok
