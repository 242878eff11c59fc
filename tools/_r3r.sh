# band kernel: which barrier removals pay (bandold = HEAD band kernel; lib = all removals)
mkdir -p gpurun_out/r3r
for v in bandold b10 drain inplace inplace_drain; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3r/kbench.jsonl || exit 1
done
timeout -k 10 300 python -u tools/kbench.py all 128 16 >> gpurun_out/r3r/kbench.jsonl || exit 1
cut -c1-200 gpurun_out/r3r/kbench.jsonl
