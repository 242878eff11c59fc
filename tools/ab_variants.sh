#!/bin/bash
# A/B the variants/*/libalifmm.so builds on the GPU box: bench line (no profiling) and the fields of
# tools/compare_libs.py per variant, then bit-identity of every variant against the first one.
# usage: tools/ab_variants.sh [bench args...]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
first=""
for d in variants/*/; do
  n=$(basename $d)
  export ALIFMM_LIB=$PWD/$d/libalifmm.so
  timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/ab/$n.bench 2>&1 || { echo "variant $n bench failed"; tail -5 gpurun_out/ab/$n.bench; exit 1; }
  timeout -k 10 120 python tools/compare_libs.py run gpurun_out/ab/$n.npz > gpurun_out/ab/$n.cmp 2>&1 || { echo "variant $n fields failed"; tail -5 gpurun_out/ab/$n.cmp; exit 1; }
  echo "$n $(python -c "import json; d=json.loads(open('gpurun_out/ab/$n.bench').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],1), d['kernel_ms_per_step'], round(d['value']/1e9,3))")"
  [ -z "$first" ] && first=$n || python tools/compare_libs.py compare gpurun_out/ab/$first.npz gpurun_out/ab/$n.npz
done
rm -f gpurun_out/ab/*.npz  # field dumps are large; only the verdicts travel back
unset ALIFMM_LIB
