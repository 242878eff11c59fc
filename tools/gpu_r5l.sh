#!/bin/bash
# ray tracer: material-id window per step (rwin1) vs per-piece loads (rwin0): C5 full + share, identity
set -o pipefail
mkdir -p gpurun_out/r5l
for v in rwin0 rwin1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5l/$v.npz > gpurun_out/r5l/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5l/${v}_share.npz > gpurun_out/r5l/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
    a,b=np.load('gpurun_out/r5l/rwin0%s.npz'%s),np.load('gpurun_out/r5l/rwin1%s.npz'%s)
    print(s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5l/ident.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5l/pytest.log 2>&1
