mkdir -p gpurun_out/r3d
for v in none nowpe nofar cur; do echo -n "$v "; ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 100 python -u tools/coop_check.py 1 16 | tail -1 || exit 1; done
