#!/bin/bash
# Counter passes for one render (run on the GPU box from the repo root).
# usage: tools/pmc.sh <outdir> <prof_one args...>
export TMPDIR=/tmp
out=$1; shift
set -e
rocprofv3 -L > gpurun_out/$out.counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/$out/p$i -o run --output-format csv -- python3 tools/prof_one.py "$@"
done
