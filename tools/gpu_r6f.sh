set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "golden_c2 or inplace or boundary or oracle_gpu or lifecycle or dropin" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; tail -5 $O/pytest.log; exit 11; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/stamps_batched.py 65536 > $O/stamps.out 2> $O/stamps.txt || { echo "stamps failed"; tail -5 $O/stamps.txt; exit 12; }
tail -5 $O/stamps.txt
timeout -k 10 300 python -c "
import json, torch, bench
dev = torch.device('cuda:0')
print(json.dumps({k: bench.bench_dropin(dev, k, c, oracle=False) for k, c in (('c1', 200), ('c2', 30))}))
" > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; tail -5 $O/dropin.err; exit 13; }
python3 -c "
import json; d=json.load(open('$O/dropin.json'))
for k in d: print(k, round(d[k]['latency_ms'],3), d[k]['split_ms'], d[k].get('libpcx_stage_ms'))"
