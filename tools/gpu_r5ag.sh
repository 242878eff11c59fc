#!/bin/bash
# init walk: the next pop classified and handed over before the last sift-up of the current one
# (ea1) vs after it (ea0): kbench 128 / 16 sources (init ms, fields fingerprint), C3; GPU tests
set -o pipefail
O=gpurun_out/r5ag
mkdir -p $O
for v in ea0 ea1 ea0 ea1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/c3.jsonl 2>>$O/$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
