#!/bin/bash
# VALU-issue bound of the bench's render kernel (C2, the contiguous instance bench.py times at N = 1,
# jump tables on): one counter pass with the kernel trace, then
# tools/valu_summary.py writes the per-launch summary bench.py reads
# (profiles/valu_c2.json).  usage: tools/pmc_valu.sh <outdir>
export TMPDIR=/tmp
out=$1
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace \
  -d "$out" -o run --output-format csv -- python3 tools/quick_bench.py --spp 1000 --reps 2 > "$out/run.log" 2>&1
