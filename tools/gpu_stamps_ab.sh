# Per-phase shader clocks of the batched kernel at low occupancy (B rounds), for several builds.
# usage: gpurun -- 'bash tools/gpu_stamps_ab.sh TAG B LIB...'
set -o pipefail
TAG=$1; B=$2; shift 2
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for L in "$@"; do
  PCX_LIB=$L timeout -k 10 100 python tools/stamps_batched.py $B > $O/s.log 2>&1 || { echo "stamps rc=$?"; tail -3 $O/s.log; exit 1; }
  echo "$L $(grep PCX_STAMPS $O/s.log | tail -1 | sed 's/PCX_STAMPS mean cycles per phase://')"
done
