#!/bin/bash
# ray kernel: the marginal cost of the group-velocity evaluations (dbl: each evaluated twice,
# same rays) vs base; C5 full, identity
set -o pipefail
mkdir -p gpurun_out/r5u
for v in base dbl base dbl; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5u/$v.npz >> gpurun_out/r5u/$v.json 2>&1 || exit 1
done
python -c "
import numpy as np
a,b=np.load('gpurun_out/r5u/base.npz'),np.load('gpurun_out/r5u/dbl.npz')
print('identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5u/ident.txt
