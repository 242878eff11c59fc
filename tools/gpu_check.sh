#!/bin/bash
# One GPU-box round of checks (run from the repo root through gpurun):
#   tools/gpu_check.sh TAG [tests|smoke|bench|stats]...   (default: all four, in that order)
# tests: pytest -m gpu (per-test timeout); smoke: __graft_entry__.smoke(); bench: bench.py line;
# stats: one rocprofv3 --kernel-trace --stats pass over a 1-step bench whose exit status is checked
# (round 2's profiled runs ended in SIGSEGV at exit).  Every step has its own time limit and the
# script stops at the first failure.
TAG=$1; shift
STEPS=${*:-tests smoke bench stats}
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
           tail -2 $OUT/smoke.log ;;
    bench) timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1; rc=$?; grep '"metric"' $OUT/bench.log | tail -1 ;;
    stats) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stats -o run \
             -- python3 $ROOT/bench.py --no-cpu --no-return --no-e2e --steps 1 --warmup 0 > $OUT/prof_stats.log 2>&1)
           rc=$?; echo "rocprofv3 exit status $rc"; ls $OUT/prof_stats/*/ 2>/dev/null | head ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $s failed: $rc"; exit $rc; fi
done
echo "== done $(date +%T)"
