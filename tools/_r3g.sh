mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "members or c4_full" > gpurun_out/r3g/tests_w1.log 2>&1; rc=$?; tail -3 gpurun_out/r3g/tests_w1.log; [ $rc -eq 0 ] || exit $rc
for v in w1 w3; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 | tail -1 || exit 1; done
ALIFMM_LIB=$PWD/variants/w3/libalifmm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "members or c4_full or c4_4096 or weld or small" > gpurun_out/r3g/tests_w3.log 2>&1; rc=$?; tail -3 gpurun_out/r3g/tests_w3.log; exit $rc
