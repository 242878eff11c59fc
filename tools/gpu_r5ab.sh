#!/bin/bash
# (1) ray tracer: piece lengths kept in LDS for the summing walk (pc12 / pc8 pieces) vs walking
#     again (base): C5 full + share, identity;
# (2) init / exact walks: a changed entry's stage decided unchanged from the changed slots alone
#     (stage_unchanged_lanes; pc12) vs re-running the stage (fs0): kbench 128 / 16 (init ms, fields
#     fingerprint), C3, weld subgrid 9; the per-pop diagnostic build (dg1);
# (3) set_model timing; the GPU tests on the in-tree build (pc12)
set -o pipefail
O=gpurun_out/r5ab
mkdir -p $O
for v in base pc12 pc8; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump $O/$v.npz > $O/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump $O/${v}_share.npz > $O/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
  a=np.load('$O/base%s.npz'%s)
  for v in ('pc12', 'pc8'):
    b=np.load('$O/%s%s.npz'%(v,s))
    print(v, s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > $O/ident.txt
for v in fs0 pc12 fs0 pc12; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> $O/kbench.jsonl 2>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/c3_bench.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/c3.jsonl 2>>$O/$v.err || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/weld_split.py | sed "s/^{/{\"variant\": \"$v\", /" >> $O/weld.jsonl 2>>$O/$v.err || exit 1
done
ALIFMM_LIB=$PWD/variants/dg1/libalifmm.so timeout -k 10 200 python -u tools/init_diag.py > $O/init_diag.json 2>&1 || exit 1
timeout -k 10 120 python tools/setmodel_time.py > $O/setmodel.json 2>&1 || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
