mkdir -p gpurun_out/r3f
for v in w1 w2; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 | tail -1 || exit 1; done
