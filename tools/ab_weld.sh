#!/bin/bash
# A/B the variants/*/libalifmm.so builds on subgrid-9 weld fields (tools/weld_split.py timing) and
# bit-identity of the fields (GPU box).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abw
first=""
for d in variants/*/; do
  n=$(basename $d)
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 120 python tools/weld_split.py --dump gpurun_out/abw/$n.npz > gpurun_out/abw/$n.log 2>&1 || { echo "variant $n failed"; tail -5 gpurun_out/abw/$n.log; exit 1; }
  echo "$n $(grep wall_s gpurun_out/abw/$n.log | tail -1)"
  [ -z "$first" ] && first=$n || python -c "
import numpy as np
a, b = np.load('gpurun_out/abw/$first.npz'), np.load('gpurun_out/abw/$n.npz')
print('identical' if all(np.array_equal(a[k], b[k]) for k in a.files) else 'DIFFER')"
done
rm -f gpurun_out/abw/*.npz
