#!/bin/bash
# run a tool for every variants/*/libalifmm.so (GPU box): tools/variant_run.sh tools/X.py [args]
cd "$(dirname "$0")/.."
for d in variants/*/; do
  n=$(basename $d)
  echo -n "$n "
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 200 python "$@" | tail -1 || exit 1
done
