# GPU check of the clustering algorithms (batched kernel) + the batched parity suite.
# usage: gpurun --timeout 600 -- 'bash tools/gpu_clusters.sh TAG'
set -o pipefail
TAG=${1:-clus}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_clusters_gpu.py tests/test_batched_gpu.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
