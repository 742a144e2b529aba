# The round-end driver's own steps on the in-tree build: every GPU test, smoke, the default bench line.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-validate}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 11; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 12; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 13; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('C3', round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_ms'], d['roofline']['frac'], 'C5', round(d['c5']['latency_ms'],1), d['c5']['stage_ms']['M_SEL_HIST'], 'C4', round(d['c4']['latency_ms'],2))"
