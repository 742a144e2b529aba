# GPU pytest run without -x (collects every failure).  usage: gpurun -- 'bash tools/gpu_tests.sh TAG [pytest args...]'
set -o pipefail
TAG=${1:-tests}
shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
if [ $# -eq 0 ]; then set -- tests -m gpu; fi
timeout -k 10 1000 python -u -m pytest "$@" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -40
exit $rc
