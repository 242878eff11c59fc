#!/bin/bash
# ray tracer: material ids of a segment's first 8/12 pieces read ahead in tbp_wave (pf8, pf12) vs
# one read per piece (pf0), C5 full + share with identity; init / exact walks: update()'s finish
# out of line (pf8) vs inlined (f0): kbench 128 + 16 sources, C3, weld subgrid 9 (exact_lds)
set -o pipefail
mkdir -p gpurun_out/r5t
for v in pf0 pf8 pf12; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5t/$v.npz > gpurun_out/r5t/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5t/${v}_share.npz > gpurun_out/r5t/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
  a=np.load('gpurun_out/r5t/pf0%s.npz'%s)
  for v in ('pf8', 'pf12'):
    b=np.load('gpurun_out/r5t/%s%s.npz'%(v,s))
    print(v, s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5t/ident.txt
for v in f0 pf8 f0 pf8; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r5t/init.jsonl 2>gpurun_out/r5t/init_$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5t/init.jsonl 2>>gpurun_out/r5t/init_$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/weld_split.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5t/init.jsonl 2>>gpurun_out/r5t/init_$v.err || exit 1
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r5t/pytest.log 2>&1
