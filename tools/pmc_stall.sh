#!/bin/bash
# Where the pool kernel's wave-cycles go: issue (VALU, dual VALU, scalar, LDS,
# branch), issue stalls, waits, and the average SMEM / LDS / VMEM latency.
# One counter group per rocprofv3 pass (--kernel-trace only).  Run on the GPU
# box from the repo root.  usage: tools/pmc_stall.sh <outdir> [quick_bench args...]
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
i=0
for set in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VALU" \
           "SmemLatency" "LdsLatency" "VmemLatency"; do
  i=$((i+1))
  echo "pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$out/p$i" -o run --output-format csv \
    -- python3 tools/quick_bench.py "$@" > "$out/p$i.log" 2>&1 || exit 1
done
