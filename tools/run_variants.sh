#!/bin/bash
# Run tools/band_profile.py against every variants/*/libalifmm.so (GPU box).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/variants
for d in variants/*/; do
  n=$(basename $d)
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 120 python tools/band_profile.py "$@" > gpurun_out/variants/$n.json 2>&1 || { echo "variant $n failed"; cat gpurun_out/variants/$n.json; exit 1; }
  echo "$n $(python -c "import json,sys; d=json.load(open('gpurun_out/variants/$n.json')); print(round(d['band_ms'],1), round(d['us_per_step'],1), d['phase_ms_mean'], d['steps_mean'])")"
done
