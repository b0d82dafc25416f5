#!/bin/bash
# Build an experiment librtp variant with extra compile definitions, for
# tools/ab.sh (RTP_LIB_PATH).  usage: tools/build_variant.sh <out.so> [-DNAME=value ...]
# With RTP_SRC_REV=<git rev> the sources of that revision are built instead.
set -e
out=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/raytracingtherestofyourlife_amd/csrc
inc=$root/include
if [ -n "$RTP_SRC_REV" ]; then
  tmp=$(mktemp -d)
  git -C "$root" archive "$RTP_SRC_REV" raytracingtherestofyourlife_amd/csrc include | tar -x -C "$tmp"
  src=$tmp/raytracingtherestofyourlife_amd/csrc
fi
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize "$@" \
  -o "$out" "$src"/rtp_kernels.hip "$src"/rtp_direct.hip "$src"/rtp_bvh_gpu.hip "$src"/rtp_host.cpp \
  "$src"/rtp_direct_host.cpp "$src"/scene_cornell.cpp
[ -n "$RTP_SRC_REV" ] && rm -rf "$tmp"
echo "$out"
