mkdir -p gpurun_out/r3l
for v in brick; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3l/kbench.jsonl || exit 1; tail -1 gpurun_out/r3l/kbench.jsonl | cut -c1-400; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3l/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3l/tests.log; exit $rc
