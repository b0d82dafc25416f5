#!/bin/bash
# tools/lat_bench (and tools/lat_bench_<tag> with extra -D flags): see tools/lat_bench.hip
# usage: tools/build_lat_bench.sh [tag -DFLAG=...]
set -e
cd "$(dirname "$0")/.."
out=tools/lat_bench${1:+_$1}; shift || true
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize "$@" \
  -I raytracingtherestofyourlife_amd/csrc tools/lat_bench.hip -L raytracingtherestofyourlife_amd -lrtp \
  -Wl,-rpath,'$ORIGIN/../raytracingtherestofyourlife_amd' -o "$out"
echo "$out"
