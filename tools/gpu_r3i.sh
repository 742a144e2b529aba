export TMPDIR=/tmp; O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_matrix_gpu.py tests/test_c5_gpu.py tests/test_batched_gpu.py -q -x --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit 11; }
bash tools/gpu_c5_ab.sh r3i_ab5 ab/HEAD/libpcx.so pyconsensus_amd/libpcx.so && bash tools/gpu_ab.sh r3i_ab3 ab/HEAD/libpcx.so pyconsensus_amd/libpcx.so
