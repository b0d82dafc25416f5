#!/bin/bash
# Dynamic instruction counts per bounce part: tools/lat_bench's modes (closest
# hit, its exact scan and prefilter, shade_hit, the loop's own ray advance;
# W = 1..5 waves per SIMD) under two SQ counter passes.  tools/lat_pmc_summary.py
# divides each dispatch's counts by its waves and loop iterations: wave-level
# instructions of each kind per step, and the wave-cycles they take.
# usage: tools/pmc_lat.sh <outdir> [iters] [modes...]   (run on the GPU box from the repo root)
export TMPDIR=/tmp
out=$1; shift
iters=${1:-2000}; shift
modes=${*:-"5 0 6 7 3 1"}
mkdir -p "$out"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$out/p$i" -o run --output-format csv \
    -- tools/lat_bench "$iters" $modes > "$out/p$i.log" 2>&1 || exit 1
done
python3 tools/lat_pmc_summary.py "$out" "$iters"
