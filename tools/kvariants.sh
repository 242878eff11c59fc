#!/bin/bash
# Build library variants into variants/<name>/libalifmm.so: the sources in $KSRCS (default
# fmm_band_k.hip) get the variant's -D flags, every other object is the in-tree build's.
# usage: [KSRCS="a.hip b.hip"] tools/kvariants.sh "NAME -DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/../ali-fmm-and-ray-tracing_amd/csrc"
make -s -j8 >/dev/null
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off"
SRCS=${KSRCS:-fmm_band_k.hip}
rm -rf ../../variants; mkdir -p ../../variants
for v in "$@"; do
  set -- $v; n=$1; shift
  mkdir -p ../../variants/$n
  for s in $SRCS; do
    /opt/rocm/bin/hipcc $FLAGS "$@" -c $s -o ../../variants/$n/${s%.hip}.o &
    pids="$pids $!"
  done
done
for p in $pids; do wait $p || { echo "a variant failed to compile"; exit 1; }; done
OTHERS=$(for s in $(sed -n "s/^SRCS = //p" Makefile); do echo ../build/$s.o; done)
for s in $SRCS; do OTHERS=$(echo "$OTHERS" | grep -v "/${s}.o"); done
for d in ../../variants/*/; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libalifmm.so $OTHERS $d/*.o
done
