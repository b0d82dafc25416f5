#!/bin/bash
# Counter passes (one counter group per rocprofv3 run, --kernel-trace only;
# never combined with runtime/sys tracing).  Run on the GPU box from the repo root.
# usage: tools/pmc.sh <outname> <python script + args...>
export TMPDIR=/tmp
out=$1; shift
set -e
mkdir -p gpurun_out/$out
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/$out/p$i -o run --output-format csv -- python3 "$@"
done
