# One GPU call for a change set: an optional A/B of batched-kernel builds (ab/NAME/libpcx.so,
# alternated twice), then the whole GPU suite, one C5 shard's stage times and a short bench.
# usage: gpurun --timeout 1500 -- 'bash tools/gpu_all.sh TAG "ab/x/libpcx.so ab/y/libpcx.so" "ab/p/libpcx.so ..."'
#   (first list: C3 batched A/B; second list: C5 1-GPU latency A/B with stage times)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-all}
ABC3=${2:-}
ABC5=${3:-}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for L in $ABC5; do
    PCX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --c5-steps 3 --steps 3 > $O/c5ab.json 2> $O/c5ab.err || { echo "c5 ab rc=$? ($L)"; tail -3 $O/c5ab.err; exit 16; }
    python3 -c "import json,sys; c=json.load(open('$O/c5ab.json'))['c5']; s=c['stage_ms']; print('%-24s C5 %.1f ms ' % (sys.argv[1], c['latency_ms']) + ' '.join('%s %.2f' % (k[2:], v) for k, v in list(s.items())[:12]))" "$L"
  done
done
for i in 1 2; do
  for L in $ABC3; do
    PCX_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --c5-steps 0 --no-c4 --steps 30 > $O/ab.json 2> $O/ab.err || { echo "ab rc=$? ($L)"; tail -3 $O/ab.err; exit 15; }
    python3 -c "import json,sys; d=json.load(open('$O/ab.json')); print('%-30s %.4f ms  %.2fM rounds/s' % (sys.argv[1], d['roofline']['kernel_ms'], d['value']/1e6))" "$L"
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 11; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 13; }
python -c "import json; d=json.load(open('$O/w8.json')); print('shard', d['latency_ms'], d['stage_ms'])"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c4 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 14; }
python -c "import json,sys; d=json.load(open('$O/bench.json')); print('C3', d['value'], d['roofline']['kernel_ms'], 'C5', d['c5']['latency_ms'], d['c5']['stage_ms'])"
