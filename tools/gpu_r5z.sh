#!/bin/bash
# round-5 final evidence on the shipped library: GPU tests, the default bench line, counter passes
# (band kernel at 128 sources: stats + FETCH + WRITE + SQ; LDS exact walk on the weld example:
# stats + SQ; ray kernel on C5: stats + FETCH + WRITE + SQ).  Shares: tools/gpu_r5z_shares.sh
set -o pipefail
T=${1:-r5z}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 &&
timeout -k 10 600 bash tools/profile.sh ${T} "stats fetch write sq" &&
PROG="python3 tools/weld_split.py" timeout -k 10 300 bash tools/profile.sh ${T}exact "stats sq" &&
PROG="python3 tools/fmc_bench.py --receivers 256" timeout -k 10 600 bash tools/profile.sh ${T}rays "stats fetch write sq"
