#!/bin/bash
# Kernel time of each BASELINE.json configuration on one MI355X
# (tools/quick_bench.py, contiguous pixels, HIP-event kernel time).
# usage: tools/configs_bench.sh <outdir>
out=${1:-gpurun_out/configs}
mkdir -p "$out"
run() { name=$1; shift; timeout -k 10 300 python3 tools/quick_bench.py "$@" > "$out/$name.log" 2>&1 || exit 1; echo "$name $(grep '^{' "$out/$name.log" | tail -1)"; }
run c1 --nx 200 --ny 200 --spp 10 --depth 10 --reps 3
run c2 --nx 800 --ny 800 --spp 1000 --depth 50 --reps 2
run c3 --nx 2048 --ny 2048 --spp 256 --depth 50 --variant 3 --reps 1
run c4 --nx 1920 --ny 1080 --spp 4096 --depth 50 --reps 1
run c5_256spp --nx 3840 --ny 2160 --spp 256 --depth 50 --reps 1
