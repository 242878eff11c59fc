#!/bin/bash
# init walks: hand-off polls spinning (sl0) vs s_sleep 1 between polls (sl1)
O=gpurun_out/r5aj
mkdir -p $O
for v in sl1 sl0 sl1 sl0; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/weld_split.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/weld.jsonl 2>>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/c3.jsonl 2>>$O/$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
