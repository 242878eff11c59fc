#!/bin/bash
# init walk: the next pop classified while the last relaxation runs (pre) vs after it (prev = f1ed1f02)
O=gpurun_out/r5ai
mkdir -p $O
for v in prev pre prev pre; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/c3.jsonl 2>>$O/$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
