#!/bin/bash
# One rocprofv3 pass over the bench configuration (run on the GPU box from the repo root):
#   tools/profile.sh TAG stats|fetch|write|sq [bench args...]  ->  gpurun_out/prof_TAG/PASS/
# One pass per gpurun call: the profiled process can crash in its exit handlers after the tool
# has written its output (seen with the cooperative-launch band kernel), and nothing else should
# run on the GPU in a call after a crash.  Summarise here afterwards with
#   python3 tools/traffic.py gpurun_out/prof_TAG TAG   (-> profiles/TAG_kernel_stats.csv, TAG_traffic.json)
TAG=$1; PASS=$2; shift 2
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
case $PASS in
  stats) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/stats.log 2>&1 ;;
  fetch) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/pmc_fetch.log 2>&1 ;;
  write) timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/pmc_write.log 2>&1 ;;
  sq) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python3 $ROOT/bench.py --no-cpu "$@" > $OUT/pmc_sq.log 2>&1 ;;
  *) echo "unknown pass $PASS"; exit 2 ;;
esac
rc=$?
grep -h '"metric"' $OUT/*.log | tail -1
ls $OUT/*/ | head -20
exit $rc
