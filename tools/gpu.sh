#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r5*.sh scripts).
#   tools/gpu.sh TAG STEP [STEP ...]        (from the repo root, on the GPU box via gpurun)
# Steps (each under its own time limit; the script stops at the first failure):
#   pytest            the -m gpu suite                       -> gpurun_out/TAG_pytest.log
#   bench[:ARGS]      python bench.py ARGS (',' = space)      -> gpurun_out/TAG_bench.log
#   kbench:SIZES      tools/kbench.py on the in-tree library  -> gpurun_out/TAG/kbench.jsonl
#   kab:SIZES[:REP]   tools/kbench.py for every variants/*/libalifmm.so, REP rounds interleaved
#   prof:PASSES       tools/profile.sh TAG "PASSES" (stats fetch write sq ...; ',' = space)
#   shares            FETCH / WRITE passes at the 2 / 4 / 8-GPU shares (64 / 32 / 16 sources)
#   py:SCRIPT[:ARGS]  python tools/SCRIPT ARGS (':' = space)  -> gpurun_out/TAG/SCRIPT.log
#   vab:SCRIPT[:ARGS] the same for every variants/*/libalifmm.so (ALIFMM_LIB), last output line
#                     of each prefixed with the variant name   -> gpurun_out/TAG/vab.log
#   smoke             __graft_entry__.smoke()                  -> gpurun_out/TAG_smoke.log
# Variant builds: tools/kvariants.sh "NAME -DFLAG=..." ...; profiles of another program:
#   PROG="python3 tools/weld_split.py" tools/gpu.sh TAG prof:stats,sq
# SIZES are comma-separated source counts, e.g. kab:16,128:2
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for STEP in "$@"; do
  KIND=${STEP%%:*}; ARG=${STEP#*:}; [ "$ARG" = "$STEP" ] && ARG=""
  case $KIND in
    pytest)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        > gpurun_out/${TAG}_pytest.log 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py ${ARG//,/ } > gpurun_out/${TAG}_bench.log 2>&1 ;;
    kbench)
      timeout -k 10 300 python -u tools/kbench.py intree ${ARG//,/ } >> $O/kbench.jsonl 2> $O/kbench.err ;;
    kab)
      SIZES=${ARG%%:*}; REP=${ARG#*:}; [ "$REP" = "$ARG" ] && REP=1
      rc=0
      for r in $(seq $REP); do
        for d in variants/*/; do
          n=$(basename $d)
          ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $n ${SIZES//,/ } \
            >> $O/kbench.jsonl 2> $O/kab_$n.err || { echo "variant $n failed"; tail -5 $O/kab_$n.err; rc=1; break 2; }
        done
      done
      [ $rc -eq 0 ] ;;
    prof)
      timeout -k 10 900 bash tools/profile.sh $TAG "${ARG//,/ }" ;;
    shares)
      for s in 64 32 16; do
        timeout -k 10 400 bash tools/profile.sh ${TAG}s$s "fetch write" --sources $s || exit 1
      done ;;
    py)
      S=${ARG%%:*}; A=${ARG#*:}; [ "$A" = "$ARG" ] && A=""
      timeout -k 10 600 python -u tools/$S ${A//:/ } > $O/${S%.py}.log 2>&1 ;;
    vab)
      S=${ARG%%:*}; A=${ARG#*:}; [ "$A" = "$ARG" ] && A=""
      rc=0
      for d in variants/*/; do
        n=$(basename $d)
        out=$(ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 300 python -u tools/$S ${A//:/ } 2> $O/vab_$n.err) \
          || { echo "variant $n failed"; tail -5 $O/vab_$n.err; rc=1; break; }
        echo "$n $(echo "$out" | tail -1)" >> $O/vab.log
      done
      [ $rc -eq 0 ] ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 ;;
    *)
      echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  echo "step $STEP exit status $rc"
  [ $rc -eq 0 ] || exit $rc
done
