#!/bin/bash
# Same-box A/B of the contiguous-pixel instance (tools/quick_bench.py) and the
# tile-deal instance bench.py runs (--tiles), and the pixel-list path over the
# tile deal's order (--list-tiles) and over the contiguous order (--list-contig): interleaved rounds, best kernel
# time of 3 C2 renders each.  usage: tools/ab_tiles.sh <rounds> [librtp.so]
rounds=$1
[ -n "$2" ] && export RTP_LIB_PATH=$2
for r in $(seq 1 "$rounds"); do
  for mode in "" "--tiles" "--list-tiles" "--list-contig"; do
    ms=$(timeout -k 10 300 python3 tools/quick_bench.py --spp 1000 --reps 3 $mode | python3 -c '
import json,sys
print(min(json.loads(l)["kernel_ms"] for l in sys.stdin if l.startswith("{")))') || exit 1
    echo "round $r [${mode:-contiguous}] kernel_ms $ms"
  done
done
