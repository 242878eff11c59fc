#!/bin/bash
# init_profile.py for every variants/*/libalifmm.so (GPU box)
cd "$(dirname "$0")/.."
for d in variants/*/; do
  n=$(basename $d)
  echo -n "$n "
  ALIFMM_LIB=$PWD/$d/libalifmm.so timeout -k 10 200 python tools/init_profile.py || exit 1
done
