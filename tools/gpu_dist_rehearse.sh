# Multi-rank rehearsal on a one-GPU box: the 2-process sharded-consensus test, then
# bench.py as the driver launches it for N=2 (torch.distributed.run, one process per
# rank), with PCX_DIST_BACKEND=gloo because both ranks share cuda:0 (RCCL refuses that).
# usage: gpurun --timeout 900 -- 'bash tools/gpu_dist_rehearse.sh TAG'
set -o pipefail
TAG=${1:-dist}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_dist.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_dist.log; exit 11; }
tail -2 $O/pytest_dist.log
PCX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --c5-steps 2 \
    --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || { echo "bench2 rc=$?"; tail -30 $O/bench2.err; exit 12; }
cat $O/bench2.json
