# Single-matrix path check: GPU parity tests through pcx_consensus_f64 (+ optional pytest args).
# usage: gpurun -- 'bash tools/gpu_matrix.sh TAG [pytest args...]'
set -o pipefail
TAG=${1:-matrix}
shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
if [ $# -eq 0 ]; then set -- tests/test_matrix_gpu.py tests/test_oracle_gpu.py tests/test_dist_gpu.py; fi
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|SKIP|passed|failed" $O/pytest.log | tail -40
[ $rc -eq 0 ] || { tail -60 $O/pytest.log; exit 1; }
