#!/bin/bash
# ray tracer: piece lengths kept in LDS for the summing walk (pc12, pc8 pieces) vs walking again (pc0): C5 full + share, identity; GPU tests
set -o pipefail
mkdir -p gpurun_out/r5aa
V="pc0 pc12 pc8"
for v in $V; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5aa/$v.npz > gpurun_out/r5aa/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5aa/${v}_share.npz > gpurun_out/r5aa/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
  a=np.load('gpurun_out/r5aa/pc0%s.npz'%s)
  for v in 'pc12 pc8'.split():
    b=np.load('gpurun_out/r5aa/%s%s.npz'%(v,s))
    print(v, s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5aa/ident.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5aa/pytest.log 2>&1
