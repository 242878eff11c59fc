# init-kernel activity breakdown (diagnostic build)
mkdir -p gpurun_out/r3p
ALIFMM_LIB=$PWD/variants/idiag/libalifmm.so timeout -k 10 300 python -u tools/init_diag.py 128 > gpurun_out/r3p/init_diag.jsonl || exit 1
cat gpurun_out/r3p/init_diag.jsonl
