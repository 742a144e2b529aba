# A/B of the C3 batched bench: alternate builds in one call (same box, same clocks).
# usage: gpurun -- 'bash tools/gpu_ab.sh TAG LIB_A LIB_B [LIB_C ...]'
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for L in "$@"; do
    PCX_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --c5-steps 0 --no-c4 --steps 30 > $O/b.json 2> $O/b.err || { echo "bench rc=$? ($L)"; tail -3 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('%-40s %.3f ms  %.2fM rounds/s' % (sys.argv[1], d['roofline']['kernel_ms'], d['value']/1e6))" "$L"
  done
done
