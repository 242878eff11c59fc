#!/bin/bash
# FETCH / WRITE passes of the band kernel at the per-GPU shares of BASELINE C4 on 2 / 4 / 8 GPUs
# (64 / 32 / 16 sources), so the driver's N > 1 bench lines carry roofline.traffic too
set -o pipefail
T=${1:-r5z}
for s in 64 32 16; do
  timeout -k 10 400 bash tools/profile.sh ${T}s$s "fetch write" --sources $s || exit 1
done
