#!/bin/bash
# Build K-member band kernel variants into variants/<name>/libalifmm.so: fmm_band_k.hip gets the
# variant's -D flags, every other object is the in-tree build's.
# usage: tools/kvariants.sh "NAME -DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/../ali-fmm-and-ray-tracing_amd/csrc"
make -s -j8 >/dev/null
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off"
rm -rf ../../variants; mkdir -p ../../variants
for v in "$@"; do
  set -- $v; n=$1; shift
  mkdir -p ../../variants/$n
  /opt/rocm/bin/hipcc $FLAGS "$@" -c fmm_band_k.hip -o ../../variants/$n/fmm_band_k.o &
done
wait
OTHERS=$(ls ../build/*.o | grep -v fmm_band_k)
for d in ../../variants/*/; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libalifmm.so $OTHERS $d/fmm_band_k.o
done
