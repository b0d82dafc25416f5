#!/bin/bash
# Same-box A/B of librtp builds: interleaved rounds, best kernel time of 3
# renders each.  Workload: C2 (800x800, 1000 spp, depth 50) unless QB_ARGS
# gives other tools/quick_bench.py arguments.  Run on the GPU box from the repo root.
# usage: [QB_ARGS="..."] tools/ab.sh <rounds> lib1.so lib2.so ...   ("main" = the in-tree librtp.so)
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    if [ "$lib" = main ]; then unset RTP_LIB_PATH; else export RTP_LIB_PATH=$lib; fi
    ms=$(timeout -k 10 300 python3 tools/quick_bench.py ${QB_ARGS:---spp 1000} --reps 3 | python3 -c '
import json,sys
print(min(json.loads(l)["kernel_ms"] for l in sys.stdin if l.startswith("{")))') || exit 1
    echo "round $r $lib kernel_ms $ms"
  done
done
