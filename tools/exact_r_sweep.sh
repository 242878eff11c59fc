#!/bin/bash
# exact-prefix radius sweep (GPU box): init profile + the GPU parity tests' measured envelope per
# radius -> gpurun_out/exr_R_{init.json,envelope.json,tests.log}.  usage: tools/exact_r_sweep.sh R...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in "$@"; do
  ALIFMM_OPT_EXACT_R=$r timeout -k 10 120 python tools/init_profile.py > gpurun_out/exr_${r}_init.json || exit 1
  ALIFMM_OPT_EXACT_R=$r timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "c1_fields or weld_sg1 or c3_2048 or c4_4096 or fmm_small or weld_sg9" > gpurun_out/exr_${r}_tests.log 2>&1
  cp gpurun_out/parity_envelope.json gpurun_out/exr_${r}_envelope.json
  echo "exact_r=$r $(cat gpurun_out/exr_${r}_init.json) $(tail -1 gpurun_out/exr_${r}_tests.log)"
done
