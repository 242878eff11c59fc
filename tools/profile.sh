#!/bin/bash
# Kernel-trace stats + HBM-traffic PMC passes for the bench configuration (run on the GPU box from
# the repo root).  usage: tools/profile.sh TAG [bench args...]
#   -> gpurun_out/prof_TAG/{stats,pmc_fetch,pmc_write}/ and profiles/TAG_{kernel_stats.csv,traffic.json}
set -e
TAG=$1; shift
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT $ROOT/profiles
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/stats.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/pmc_write.log 2>&1
cd $ROOT
python3 tools/traffic.py $OUT $TAG
echo done
