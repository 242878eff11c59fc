# init kernel: square stencils of the verification on 8 lanes per job
mkdir -p gpurun_out/r3t
ALIFMM_LIB=$PWD/variants/idiag/libalifmm.so timeout -k 10 300 python -u tools/init_diag.py 128 > gpurun_out/r3t/init_diag.jsonl || exit 1
cat gpurun_out/r3t/init_diag.jsonl
timeout -k 10 300 python -u tools/kbench.py parverify 128 16 > gpurun_out/r3t/kbench.jsonl || exit 1
ALIFMM_LIB=$PWD/variants/pv0/libalifmm.so timeout -k 10 300 python -u tools/kbench.py pv0 128 16 >> gpurun_out/r3t/kbench.jsonl || exit 1
cut -c1-200 gpurun_out/r3t/kbench.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3t/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3t/tests.log; exit $rc
