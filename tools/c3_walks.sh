#!/bin/bash
# C3 (2048^2, 1000 spheres, depth 50) kernel time of the sphere-BVH walks at
# a reduced spp: the global threaded walk (default), the LDS walk
# (RTP_BVH_LDS=1), and any extra librtp builds given.  usage: tools/c3_walks.sh <spp> [lib.so ...]
spp=$1; shift
run() { timeout -k 10 300 python3 tools/quick_bench.py --nx 2048 --ny 2048 --spp "$spp" --variant 3 --reps 2 | python3 -c '
import json,sys
print(min(json.loads(l)["kernel_ms"] for l in sys.stdin if l.startswith("{")))'; }
echo "global $(run)" || exit 1
echo "lds $(RTP_BVH_LDS=1 run)" || exit 1
for lib in "$@"; do echo "$lib $(RTP_LIB_PATH=$lib run)" || exit 1; done
