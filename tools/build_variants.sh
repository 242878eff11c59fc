#!/bin/bash
# Build band-kernel variants (tuning experiments) into variants/<name>/libalifmm.so: the band
# kernels (fmm_band.hip, fmm_band_pair.hip) get the variant's -D flags, the rest is shared.
# usage: tools/build_variants.sh "NAME -DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/../ali-fmm-and-ray-tracing_amd/csrc"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off"
mkdir -p ../build
for f in api.cpp fmm_init.hip fmm_exact.hip rays.hip utils.hip; do
  [ ../build/$f.o -nt $f ] || /opt/rocm/bin/hipcc $FLAGS -c $f -o ../build/$f.o
done
for v in "$@"; do
  set -- $v; n=$1; shift
  mkdir -p ../../variants/$n
  /opt/rocm/bin/hipcc $FLAGS "$@" -c fmm_band.hip -o ../../variants/$n/fmm_band.o &
  /opt/rocm/bin/hipcc $FLAGS "$@" -c fmm_band_pair.hip -o ../../variants/$n/fmm_band_pair.o &
done
wait
for d in ../../variants/*/; do
  [ -f $d/fmm_band.o ] && /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libalifmm.so ../build/api.cpp.o \
    ../build/fmm_init.hip.o ../build/fmm_exact.hip.o ../build/rays.hip.o ../build/utils.hip.o $d/fmm_band.o $d/fmm_band_pair.o
done
