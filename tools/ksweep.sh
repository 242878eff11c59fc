#!/bin/bash
# K / stripe sweep for 16 sources (GPU box)
cd /root/repo
for cfg in "16 4" "16 5" "8 4" "8 5" "8 6" "4 6"; do
  set -- $cfg
  ALIFMM_OPT_MEMBERS=$1 ALIFMM_OPT_STRIPE_LOG=$2 timeout -k 10 120 python -u tools/kbench.py "K$1_w$2" 16 >> gpurun_out/ksweep.jsonl || exit 1
done
