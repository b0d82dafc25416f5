#!/bin/bash
# One SQ/GRBM counter pass of a tools/quick_bench.py render (any arguments),
# for a quick bound check: VALU issue vs capacity, lanes per instruction,
# memory instructions, waiting.  usage: tools/pmc_quick.sh <outdir> [quick_bench args...]
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$out" -o run --output-format csv \
  -- python3 tools/quick_bench.py "$@" > "$out/run.log" 2>&1
