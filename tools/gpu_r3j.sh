# matrix + batched GPU tests, then the C5 and C3 A/B against HEAD and one 8-GPU shard's latency
export TMPDIR=/tmp; O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_matrix_gpu.py tests/test_c5_gpu.py tests/test_batched_gpu.py -q -x --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit 11; }
bash tools/gpu_c5_ab.sh r3j_ab5 ab/HEAD/libpcx.so pyconsensus_amd/libpcx.so || exit 12
bash tools/gpu_ab.sh r3j_ab3 ab/HEAD/libpcx.so pyconsensus_amd/libpcx.so || exit 13
timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 14; }
python3 -c "import json; d=json.load(open('$O/w8.json')); print('shard', round(d['latency_ms'],2), list(d['stage_ms'].items())[:12])"
