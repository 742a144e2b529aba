# a batched-kernel variant: its bit-exactness tests through PCX_LIB, then the C3 A/B against HEAD
export TMPDIR=/tmp; O=gpurun_out/r3m; mkdir -p $O
V=${1:-ab/cert/libpcx.so}
PCX_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_batched_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit 11; }
bash tools/gpu_ab.sh r3m_ab3 ab/HEAD/libpcx.so $V
