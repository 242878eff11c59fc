# init kernel: register-resident speculative entries; band kernel: five fewer barriers per step
mkdir -p gpurun_out/r3q
ALIFMM_LIB=$PWD/variants/idiag/libalifmm.so timeout -k 10 300 python -u tools/init_diag.py 128 > gpurun_out/r3q/init_diag.jsonl || exit 1
cat gpurun_out/r3q/init_diag.jsonl
timeout -k 10 300 python -u tools/kbench.py new 128 16 > gpurun_out/r3q/kbench.jsonl || exit 1
ALIFMM_LIB=$PWD/variants/bandold/libalifmm.so timeout -k 10 300 python -u tools/kbench.py bandold 128 16 >> gpurun_out/r3q/kbench.jsonl || exit 1
cut -c1-330 gpurun_out/r3q/kbench.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3q/tests.log; exit $rc
