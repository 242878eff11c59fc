#!/bin/bash
# ray tracer: group-velocity evaluation out of line (s1) vs inlined (s0), 2/3/4 waves per SIMD: C5 full + share, identity; GPU tests
set -o pipefail
mkdir -p gpurun_out/r5q
V="s0w2 s1w2 s1w3 s1w4"
for v in $V; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5q/$v.npz > gpurun_out/r5q/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5q/${v}_share.npz > gpurun_out/r5q/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
  a=np.load('gpurun_out/r5q/s0w2%s.npz'%s)
  for v in 's1w2 s1w3 s1w4'.split():
    b=np.load('gpurun_out/r5q/%s%s.npz'%(v,s))
    print(v, s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5q/ident.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5q/pytest.log 2>&1
