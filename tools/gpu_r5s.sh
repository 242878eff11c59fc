#!/bin/bash
# ray kernel cost split (diagnostic builds, wrong rays): without the group-velocity evaluations
# (dslo), without the material-id loads (dnoid), both, without the ray-time pass (dnotime); C5 full
set -o pipefail
mkdir -p gpurun_out/r5s
for v in base dslo dnoid dboth dnotime; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 > gpurun_out/r5s/$v.json 2>&1 || exit 1
done
