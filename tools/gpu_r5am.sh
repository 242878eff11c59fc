#!/bin/bash
# band kernel: claim items per lane per pass 1 (shipped) / 2 / 3: kbench 128 / 64 / 16 sources
# (band ms, fields fingerprint)
set -o pipefail
O=gpurun_out/r5am
mkdir -p $O
for v in u1 u2 u3 u1 u2 u3; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 64 16 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
done
