#!/bin/bash
# A/B runner (GPU box): for each variant name in $1 (space-separated; variants/<name>/libalifmm.so),
# run the rest of the command line with ALIFMM_LIB pointing at it; each output line is prefixed
# with the variant name -> stdout.  Stops at the first failure.
cd "$(dirname "$0")/.."
names=$1; shift
for n in $names; do
  out=$(ALIFMM_LIB=$PWD/variants/$n/libalifmm.so timeout -k 10 300 "$@" 2>/tmp/ab_$n.err) || { echo "variant $n failed"; tail -5 /tmp/ab_$n.err; exit 1; }
  echo "$out" | sed "s/^/$n /"
done
