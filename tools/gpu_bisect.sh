# Run a pytest selection against several libpcx builds (PCX_LIB), one line per build.
# usage: gpurun -- 'bash tools/gpu_bisect.sh TAG "PYTEST ARGS" LIB_A LIB_B ...'
set -o pipefail
TAG=$1; ARGS=$2; shift 2
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for L in "$@"; do
  n=$(echo $L | tr '/' '_')
  PCX_LIB=$L timeout -k 10 300 python -u -m pytest $ARGS -q --timeout 250 --timeout-method thread -p no:cacheprovider > $O/$n.log 2>&1
  rc=$?
  echo "$L rc=$rc $(grep -E 'passed|failed' $O/$n.log | tail -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
