#!/bin/bash
# Kernel time of rank r's share of the C4 frame (1920x1080, 4096 spp, depth 50)
# under the N-rank 16x16 tile deal through the tile instance bench.py runs
# (rtp_render_tiles_device: 1080 rows are 67.5 tiles, the clipped edge tiles
# are rendered whole; LIST=1: the pixel-list path, shard.tile_pixels), for
# N = 1, 2, 4, 8 and the first and last rank.
# usage: tools/c4_shares.sh [worlds] [spp]
worlds=${1:-"1 2 4 8"}
spp=${2:-4096}
for n in $worlds; do
  for r in $(printf "%s\n" 0 $((n - 1)) | sort -un); do
    line=$(timeout -k 10 300 python3 tools/quick_bench.py $([ "$LIST" = 1 ] && echo --share || echo --tiles) --nx 1920 --ny 1080 --spp "$spp" --depth 50 \
           --world "$n" --rank "$r" --reps 2 | grep '^{' | tail -1) || exit 1
    echo "world $n rank $r $line"
  done
done
