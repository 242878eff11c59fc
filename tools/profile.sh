#!/bin/bash
# rocprofv3 passes over the bench configuration (run on the GPU box from the repo root):
#   tools/profile.sh TAG "stats fetch write sq" [bench args...]  ->  gpurun_out/prof_TAG/PASS/
# or over another program: PROG="python3 tools/c3_bench.py" tools/profile.sh TAG "stats fetch write"
# One process per pass (PMC passes never combine with tracing domains); every pass has its own
# time limit and the script stops at the first failure.  Summarise here afterwards with
#   python3 tools/traffic.py gpurun_out/prof_TAG TAG [KERNEL]
#   (-> profiles/TAG_kernel_stats.csv, TAG_traffic.json for KERNEL, default fmm_band_k_kernel)
TAG=$1; PASSES=$2; shift 2
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
if [ -n "$PROG" ]; then
  B=$(echo "$PROG" | sed "s|tools/|$ROOT/tools/|")
else
  B="python3 $ROOT/bench.py --no-cpu --no-return --no-e2e --no-c3 --no-c5"
fi
for PASS in $PASSES; do
  case $PASS in
    stats) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B "$@" > $OUT/stats.log 2>&1 ;;
    fetch) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B "$@" > $OUT/pmc_fetch.log 2>&1 ;;
    write) timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B "$@" > $OUT/pmc_write.log 2>&1 ;;
    sq) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- $B "$@" > $OUT/pmc_sq.log 2>&1 ;;
    sq2) timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $OUT/pmc_sq2 -o run -- $B "$@" > $OUT/pmc_sq2.log 2>&1 ;;
    sq3) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_CVT --output-format csv -d $OUT/pmc_sq3 -o run -- $B "$@" > $OUT/pmc_sq3.log 2>&1 ;;
    ta) timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_ta -o run -- $B "$@" > $OUT/pmc_ta.log 2>&1 ;;
    list) timeout -s KILL 120 rocprofv3 -L > $OUT/list.txt 2>&1 ;;
    ic) timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $OUT/pmc_ic -o run -- $B "$@" > $OUT/pmc_ic.log 2>&1 ;;
    ic2) timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/pmc_ic2 -o run -- $B "$@" > $OUT/pmc_ic2.log 2>&1 ;;
    calib) timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_calib -o run -- $ROOT/tools/micro/fetch_calib > $OUT/pmc_calib.log 2>&1 ;;
    wcalib) timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_wcalib -o run -- $ROOT/tools/micro/write_calib > $OUT/pmc_wcalib.log 2>&1 ;;
    *) echo "unknown pass $PASS"; exit 2 ;;
  esac
  rc=$?
  echo "pass $PASS exit status $rc"
  [ $rc -eq 0 ] || exit $rc
done
grep -h '^{' $OUT/*.log | tail -1 | cut -c1-300 || true
