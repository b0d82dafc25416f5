#!/bin/bash
# Rehearse raytracingtherestofyourlife_amd.render_dist with N ranks sharing GPU 0
# (gloo host reduce) and --check.  usage: tools/render_dist_rehearsal.sh <ranks> <shard> [render_dist args...]
n=$1; shard=$2; shift 2
RTP_FF_TABLES=${RTP_FF_TABLES:-1} exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
  --master-addr 127.0.0.1 --master-port $((29700 + n)) -m raytracingtherestofyourlife_amd.render_dist \
  --shard "$shard" --backend gloo --share-gpu --check "$@"
