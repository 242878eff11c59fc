#!/bin/bash
# run tools/kbench.py for every variants/*/libalifmm.so (GPU box); args: source counts
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in variants/*/; do
  n=$(basename $d)
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $n "$@" >> gpurun_out/kab.jsonl 2>gpurun_out/kab_$n.err || { echo "variant $n failed"; tail -5 gpurun_out/kab_$n.err; exit 1; }
done
