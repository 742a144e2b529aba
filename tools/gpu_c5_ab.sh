# A/B of the C5 latency (1 GPU) for several libpcx builds, alternating on one box.
# usage: gpurun -- 'bash tools/gpu_c5_ab.sh TAG LIB_A LIB_B [...]'
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for L in "$@"; do
    PCX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --c5-steps 3 --steps 3 > $O/b.json 2> $O/b.err || { echo "bench rc=$? ($L)"; tail -3 $O/b.err; exit 1; }
    python3 -c "import json,sys; c=json.load(open('$O/b.json'))['c5']; s=c['stage_ms']; print('%-24s C5 %.1f ms ' % (sys.argv[1], c['latency_ms']) + ' '.join('%s %.1f' % (k[2:], v) for k, v in list(s.items())[:9]))" "$L"
  done
done
