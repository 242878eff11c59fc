#!/bin/bash
# band width cdelta: GPU tests at 0.6 (parity envelope), finer sweep with kbench shares
set -o pipefail
mkdir -p gpurun_out
ALIFMM_OPT_CDELTA=0.6 timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r5h_pytest06.log 2>&1 ; echo "pytest 0.6 exit $?" >> gpurun_out/r5h_pytest06.log
cp gpurun_out/parity_envelope.json gpurun_out/r5h_parity_envelope06.json 2>/dev/null
timeout -k 10 300 python -u tools/cdelta_sweep.py 0.55 0.65 0.7 > gpurun_out/r5h_cdelta.txt 2>&1 &&
for c in 0.55 0.65 0.7; do ALIFMM_OPT_CDELTA=$c timeout -k 10 300 python -u tools/kbench.py cd$c 128 32 16 >> gpurun_out/r5h_kbench.jsonl 2>&1 || exit 1; done
