#!/bin/bash
# round-5 first GPU call: GPU tests, the default bench line (C4 + C3 sub-object), the launcher
# rehearsal (2 ranks on one device) and its refusal, kbench shares, counter passes of this build
set -o pipefail
T=${1:-r5a}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 &&
ALIFMM_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --no-cpu --no-e2e --no-return > gpurun_out/${T}_bench2.log 2>&1 &&
{ timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > gpurun_out/${T}_bench2_refuse.log 2>&1; echo "exit status $?" >> gpurun_out/${T}_bench2_refuse.log; true; } &&
timeout -k 10 300 python -u tools/kbench.py base 128 64 32 16 > gpurun_out/${T}_kbench.jsonl 2>&1 &&
timeout -k 10 900 bash tools/profile.sh ${T} "stats fetch write sq"
