mkdir -p gpurun_out/r3c
for c in 1 0; do timeout -k 10 120 python -u tools/coop_check.py $c 16 >> gpurun_out/r3c/coop.jsonl || exit 1; tail -1 gpurun_out/r3c/coop.jsonl; done
