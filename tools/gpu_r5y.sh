#!/bin/bash
# init walk: the relax role refreshes its changed speculative entries while it waits for the next
# pop (rf1) vs re-checks in turn only (rf0): kbench 128 / 16 sources (init ms, fields fingerprint),
# C3; then the GPU tests (in-tree = rf1)
set -o pipefail
mkdir -p gpurun_out/r5y
for v in rf0 rf1 rf0 rf1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> gpurun_out/r5y/kbench.jsonl 2>gpurun_out/r5y/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5y/c3.jsonl 2>>gpurun_out/r5y/$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5y/pytest.log 2>&1
