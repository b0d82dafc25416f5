#!/bin/bash
# Kernel time of one rank's share of a frame under the strong-scaling tile
# deal (rank 0 of N), for each RTP_WAVE_PIXELS value given ("default": the
# library's own choice).  Frame: C2 through the in-kernel tile deal unless
# QB_ARGS gives other tools/quick_bench.py arguments (e.g. C4:
# QB_ARGS="--share --nx 1920 --ny 1080 --spp 4096", the pixel-list path).
# usage: [QB_ARGS=...] tools/share_sweep.sh "<worlds>" "<wave_pixels values>"
for n in $1; do
  for wp in $2; do
    if [ "$wp" = default ]; then unset RTP_WAVE_PIXELS; else export RTP_WAVE_PIXELS=$wp; fi
    ms=$(timeout -k 10 300 python3 tools/quick_bench.py ${QB_ARGS:---tiles --spp 1000} --world "$n" --rank 0 --reps 2 | python3 -c '
import json,sys
print(min(json.loads(l)["kernel_ms"] for l in sys.stdin if l.startswith("{")))') || exit 1
    echo "world $n wave_pixels $wp kernel_ms $ms"
  done
done
