# round-4 evidence passes for the kernels other than the band kernel:
# C3 (BASELINE config 3) kernel stats + FETCH/WRITE + SQ, find_ray_kernel on the C5 share,
# fmm_exact_kernel on the weld example (sg 9).  Usage: bash tools/r4_prof.sh TAG
set -o pipefail
T=${1:-r4p}
PROG="python3 tools/c3_bench.py" timeout -k 10 600 bash tools/profile.sh ${T}c3 "stats fetch write sq" &&
PROG="python3 tools/fmc_bench.py" timeout -k 10 600 bash tools/profile.sh ${T}rays "stats sq" &&
PROG="python3 tools/weld_split.py" timeout -k 10 600 bash tools/profile.sh ${T}exact "stats sq"
