set -o pipefail
mkdir -p gpurun_out/r3b
bash tools/gpu_check.sh r3b stats || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_host_paths.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r3b/tests_c5.log 2>&1; rc=$?; tail -3 gpurun_out/r3b/tests_c5.log; [ $rc -eq 0 ] || exit $rc
for v in w1 w2; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3b/kbench.jsonl 2>gpurun_out/r3b/kbench_$v.err || exit 1
  tail -1 gpurun_out/r3b/kbench.jsonl
done
ALIFMM_LIB=$PWD/variants/w2/libalifmm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "members or c4_full or c4_4096 or weld or small" > gpurun_out/r3b/tests_w2.log 2>&1; rc=$?; tail -3 gpurun_out/r3b/tests_w2.log; exit $rc
