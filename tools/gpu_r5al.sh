#!/bin/bash
# LDS exact walk (subgrid > 1): the next pop classified and handed over before the current pop's
# last addtree / updtree (xe1) vs after it (xe0): weld subgrid 9 init, fields bit-identity (dump);
# then the GPU tests on the in-tree build (xe1)
set -o pipefail
O=gpurun_out/r5al
mkdir -p $O
for v in xe0 xe1 xe0 xe1; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/weld_split.py --dump $O/$v.npz | sed "s/^{/{\"variant\": \"$v\", /" >> $O/weld.jsonl 2>>$O/$v.err || exit 1
done
python -c "
import numpy as np
a,b=np.load('$O/xe0.npz'),np.load('$O/xe1.npz')
print('identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER', a.files)" > $O/ident.txt
rm -f $O/*.npz
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
