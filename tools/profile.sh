#!/bin/bash
# Kernel-trace stats + PMC passes for one bench configuration (run on the GPU box from the repo root).
# usage: tools/profile.sh TAG [bench args...]   -> gpurun_out/prof_TAG/{stats,pmc_*}
set -e
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --no-cpu "$@" > $OUT/stats.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_sq.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_misc -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_misc.log 2>&1
echo done
