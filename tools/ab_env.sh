#!/bin/bash
# Same-box A/B of environment settings for the in-tree librtp: interleaved
# rounds, best kernel time of 3 C2 renders each (QB_ARGS overrides).
# usage: tools/ab_env.sh <rounds> "VAR=val ..." "VAR=val ..." ...   ("-" = no extra variables)
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for setting in "$@"; do
    vars=""; [ "$setting" != "-" ] && vars="$setting"
    ms=$(env $vars timeout -k 10 300 python3 tools/quick_bench.py ${QB_ARGS:---spp 1000} --reps 3 | python3 -c '
import json,sys
print(min(json.loads(l)["kernel_ms"] for l in sys.stdin if l.startswith("{")))') || exit 1
    echo "round $r [$setting] kernel_ms $ms"
  done
done
