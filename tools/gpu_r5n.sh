#!/bin/bash
# ray tracer: material ids of a segment's first pieces read ahead (pf4/8/12) vs one dependent read
# per piece (pf0): C5 full + share, identity; then the GPU tests on the in-tree build
set -o pipefail
mkdir -p gpurun_out/r5n
V="pf0 pf4 pf8 pf12"
for v in $V; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5n/$v.npz > gpurun_out/r5n/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5n/${v}_share.npz > gpurun_out/r5n/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
  a=np.load('gpurun_out/r5n/pf0%s.npz'%s)
  for v in 'pf4 pf8 pf12'.split():
    b=np.load('gpurun_out/r5n/%s%s.npz'%(v,s))
    print(v, s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5n/ident.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5n/pytest.log 2>&1
