#!/bin/bash
# A/B the variants/*/libalifmm.so builds on the ray tracer (GPU box): tools/fmc_bench.py (one GPU's
# C5 share: 32 receiver fields + 8192 rays) per variant, then bit-identity of the ray times/lengths.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abr
first=""
for d in variants/*/; do
  n=$(basename $d)
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 120 python tools/fmc_bench.py --dump gpurun_out/abr/$n.npz "$@" > gpurun_out/abr/$n.json 2>&1 || { echo "variant $n failed"; tail -5 gpurun_out/abr/$n.json; exit 1; }
  echo "$n $(tail -1 gpurun_out/abr/$n.json)"
  [ -z "$first" ] && first=$n || python -c "
import numpy as np, sys
a, b = np.load('gpurun_out/abr/$first.npz'), np.load('gpurun_out/abr/$n.npz')
print('identical' if all(np.array_equal(a[k], b[k]) for k in a.files) else 'DIFFER')"
done
