mkdir -p gpurun_out/r3n
for v in base cu1 cu4 sort0 sort128 bfirst t1024; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3n/kbench.jsonl || exit 1; tail -1 gpurun_out/r3n/kbench.jsonl | cut -c1-120; done
