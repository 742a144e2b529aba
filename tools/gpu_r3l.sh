# a selection variant: matrix-path GPU tests through PCX_LIB, then the C5 A/B against HEAD
export TMPDIR=/tmp; O=gpurun_out/r3l; mkdir -p $O
V=${1:-ab/hn32/libpcx.so}
PCX_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_matrix_gpu.py tests/test_c5_gpu.py -q -x --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit 11; }
bash tools/gpu_c5_ab.sh r3l_ab5 ab/HEAD/libpcx.so $V
