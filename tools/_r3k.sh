mkdir -p gpurun_out/r3k
for v in brick rowm; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3k/kbench.jsonl || exit 1; tail -1 gpurun_out/r3k/kbench.jsonl | cut -c1-330; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3k/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3k/tests.log; exit $rc
