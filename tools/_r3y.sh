# 16-source share (K = 16): stripe width and member count
mkdir -p gpurun_out/r3y
timeout -k 10 200 python -u tools/kbench.py base 16 >> gpurun_out/r3y/kbench.jsonl || exit 1
ALIFMM_OPT_STRIPE_LOG=3 timeout -k 10 200 python -u tools/kbench.py w8 16 >> gpurun_out/r3y/kbench.jsonl || exit 1
ALIFMM_OPT_STRIPE_LOG=5 timeout -k 10 200 python -u tools/kbench.py w32 16 >> gpurun_out/r3y/kbench.jsonl || exit 1
ALIFMM_OPT_MEMBERS=12 timeout -k 10 200 python -u tools/kbench.py k12 16 >> gpurun_out/r3y/kbench.jsonl || exit 1
ALIFMM_OPT_STRIPE_LOG=5 timeout -k 10 200 python -u tools/kbench.py w32_128 128 >> gpurun_out/r3y/kbench.jsonl || exit 1
cut -c1-160 gpurun_out/r3y/kbench.jsonl
