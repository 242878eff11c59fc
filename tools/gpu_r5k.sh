#!/bin/bash
# round-5 secondary numbers on the current library: two contexts' streaming (advice item), the
# weld example end to end, the C5 share and capture timings, the init profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_multi.py > gpurun_out/r5k_stream_multi.json 2>&1 &&
timeout -k 10 300 python -u tools/weld_e2e.py > gpurun_out/r5k_weld_e2e.json 2>&1 &&
timeout -k 10 300 python -u tools/fmc_bench.py > gpurun_out/r5k_fmc_share.json 2>&1 &&
timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 > gpurun_out/r5k_fmc_full.json 2>&1 &&
timeout -k 10 300 python -u tools/init_profile.py > gpurun_out/r5k_init_profile.json 2>&1 &&
timeout -k 10 300 python -u tools/c3_bench.py > gpurun_out/r5k_c3.json 2>&1
