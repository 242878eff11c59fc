#!/bin/bash
# init-kernel A/B over variants/*/libalifmm.so (GPU box): kbench at the given source counts (band
# and init ms, fields fingerprint) and the C3 line, one JSON line each -> gpurun_out/init_ab2.jsonl
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in variants/*/; do
  n=$(basename $d)
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $n "$@" >> gpurun_out/init_ab2.jsonl 2>gpurun_out/init_ab2_$n.err || { echo "variant $n failed"; tail -5 gpurun_out/init_ab2_$n.err; exit 1; }
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$n\", /" >> gpurun_out/init_ab2.jsonl 2>>gpurun_out/init_ab2_$n.err || { echo "variant $n c3 failed"; exit 1; }
done
