#!/bin/bash
# Kernel time of rank r's share of the C5 frame (3840x2160, 16384 spp, depth
# 50) under the N-rank sample-batch shard bench.py runs at N > 1: spp/N
# samples of every pixel on the derived stream seed = pixel + r*nx*ny
# (shard.sample_batches), the contiguous work-stealing launch, for N = 1, 2,
# 4, 8 and the first and last rank.  (The C4 tile shares: tools/c4_shares.sh.)
# usage: tools/c5_shares.sh [worlds] [spp]
worlds=${1:-"1 2 4 8"}
spp=${2:-16384}
npix=$((3840 * 2160))
for n in $worlds; do
  for r in $(printf "%s\n" 0 $((n - 1)) | sort -un); do
    line=$(timeout -k 10 300 python3 tools/quick_bench.py --nx 3840 --ny 2160 --spp $((spp / n)) --depth 50 \
           --seed-base $((r * npix)) --reps 1 | grep '^{' | tail -1) || exit 1
    echo "world $n rank $r $line"
  done
done
