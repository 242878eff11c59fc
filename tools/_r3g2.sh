# stripe width sweep (runtime option stripe_log), repeated base runs for the noise level
mkdir -p gpurun_out/r3g2
for v in base:0 w128:7 base2:0; do n=${v%%:*}; l=${v##*:}
  if [ $l = 0 ]; then timeout -k 10 200 python -u tools/kbench.py $n 128 >> gpurun_out/r3g2/kbench.jsonl || exit 1
  else ALIFMM_OPT_STRIPE_LOG=$l timeout -k 10 200 python -u tools/kbench.py $n 128 >> gpurun_out/r3g2/kbench.jsonl || exit 1; fi
done
for v in b16:0 w32:5 w64:6 b16b:0 w32b:5; do n=${v%%:*}; l=${v##*:}
  if [ $l = 0 ]; then timeout -k 10 200 python -u tools/kbench.py $n 16 >> gpurun_out/r3g2/kbench.jsonl || exit 1
  else ALIFMM_OPT_STRIPE_LOG=$l timeout -k 10 200 python -u tools/kbench.py $n 16 >> gpurun_out/r3g2/kbench.jsonl || exit 1; fi
done
cut -c1-120 gpurun_out/r3g2/kbench.jsonl
