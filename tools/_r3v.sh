# init kernel: next-pop prediction (the relax wavefront verifies the predicted pop's jobs early)
mkdir -p gpurun_out/r3v
ALIFMM_LIB=$PWD/variants/idiag/libalifmm.so timeout -k 10 300 python -u tools/init_diag.py 128 > gpurun_out/r3v/init_diag.jsonl || exit 1
cat gpurun_out/r3v/init_diag.jsonl
timeout -k 10 300 python -u tools/kbench.py predict 128 16 > gpurun_out/r3v/kbench.jsonl || exit 1
ALIFMM_LIB=$PWD/variants/np0/libalifmm.so timeout -k 10 300 python -u tools/kbench.py np0 128 16 >> gpurun_out/r3v/kbench.jsonl || exit 1
cut -c1-200 gpurun_out/r3v/kbench.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3v/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3v/tests.log; exit $rc
