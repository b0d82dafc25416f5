#!/bin/bash
# One SQ instruction/lane counter pass of a quick_bench render (C2 geometry, 200 spp).
# usage: tools/pmc_sq.sh <outdir> [librtp.so]
export TMPDIR=/tmp
out=$1
[ -n "$2" ] && export RTP_LIB_PATH=$2
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --kernel-trace \
  -d "$out" -o run --output-format csv -- python3 tools/quick_bench.py --spp 200 --reps 1
