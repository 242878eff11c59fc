#!/bin/bash
# band kernel: claim dedupe by acceptance stamps (st1) vs the LDS hash (st0): kbench 128 / 64 /
# 32 / 16 sources (band ms, fields fingerprint), C3, weld subgrid 9; then the GPU tests (in-tree = st1)
set -o pipefail
mkdir -p gpurun_out/r5v
for v in st0 st1 st0 st1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 64 32 16 >> gpurun_out/r5v/kbench.jsonl 2>gpurun_out/r5v/$v.err || exit 1
done
for v in st0 st1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5v/c3.jsonl 2>>gpurun_out/r5v/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/weld_split.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5v/weld.jsonl 2>>gpurun_out/r5v/$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5v/pytest.log 2>&1
