#!/bin/bash
# band kernel members of 512 vs 768 threads (the current kernel, far band on): kbench 16 / 32 /
# 64 / 128 sources (band ms, fields fingerprint)
set -o pipefail
O=gpurun_out/r5an
mkdir -p $O
for v in t768 t512 t768 t512; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 16 32 64 128 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
done
