# Round-3 closing check in one call: C5 A/B of the build variants, every GPU test, smoke, the
# default bench line, rocprofv3 kernel trace + PMC passes of the bench, one 8-GPU shard's latency.
# usage: gpurun --timeout 1200 -- 'bash tools/gpu_final_r3.sh TAG LIB...'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-final}; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for L in "$@"; do
  PCX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-c4 --c5-steps 3 --steps 3 > $O/ab.json 2> $O/ab.err || { echo "ab rc=$? ($L)"; tail -3 $O/ab.err; exit 10; }
  python3 -c "import json,sys; c=json.load(open('$O/ab.json'))['c5']; s=c['stage_ms']; print('%-22s C5 %.1f ms ' % (sys.argv[1], c['latency_ms']) + ' '.join('%s %.1f' % (k[2:], v) for k, v in list(s.items())[:9]))" "$L"
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 11; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 12; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 13; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('C3', round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_ms'], 'C5', round(d['c5']['latency_ms'],1), 'C4', round(d['c4']['latency_ms'],2))"
bash tools/gpu_profile.sh $TAG/prof || exit 14
timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 15; }
python3 -c "import json; d=json.load(open('$O/w8.json')); print('shard', round(d['latency_ms'],2))"
