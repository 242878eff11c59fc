#!/bin/bash
# round-5 checkpoint: GPU tests, bench line, weld sg 9 split, kbench shares, band-width sweep
set -o pipefail
T=${1:-r5g}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 &&
timeout -k 10 200 python -u tools/weld_split.py > gpurun_out/${T}_weld_split.txt 2>&1 &&
timeout -k 10 300 python -u tools/kbench.py base 128 64 32 16 > gpurun_out/${T}_kbench.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/cdelta_sweep.py 0.5 0.6 0.75 > gpurun_out/${T}_cdelta.txt 2>&1 &&
ALIFMM_OPT_CDELTA=0.6 timeout -k 10 300 python -u tools/kbench.py cd06 128 16 >> gpurun_out/${T}_kbench.jsonl 2>&1
