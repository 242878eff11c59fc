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
for v in rint rnoid; do ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 > gpurun_out/r5k_rays_$v.json 2>&1 || exit 1; done
bash tools/ab_run.sh "apx0 apx1" python -u tools/kbench.py x 128 16 > gpurun_out/r5k_apex_kbench.txt &&
bash tools/ab_run.sh "apx0 apx1" python -u tools/c3_bench.py > gpurun_out/r5k_apex_c3.txt &&
bash tools/ab_run.sh "apx0 apx1" python -u tools/weld_split.py > gpurun_out/r5k_apex_weld.txt
ALIFMM_LIB=$PWD/variants/w2t256/libalifmm.so timeout -k 10 300 python -u tools/kbench.py w2t256 128 64 > gpurun_out/r5k_w2t256.jsonl 2>&1
