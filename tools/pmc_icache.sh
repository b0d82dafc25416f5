#!/bin/bash
# Instruction-fetch counters of a quick_bench render (C2 geometry, 200 spp)
# for each librtp build given ("main" = the in-tree one).  One pass each.
# usage: tools/pmc_icache.sh <outdir> lib1 lib2 ...
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -k 10 60 rocprofv3 -L > "$out/avail.txt" 2>&1
for lib in "$@"; do
  if [ "$lib" = main ]; then unset RTP_LIB_PATH; tag=main; else export RTP_LIB_PATH=$lib; tag=$(basename $lib .so); fi
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace \
    -d "$out/$tag" -o run --output-format csv -- python3 tools/quick_bench.py --spp 200 --reps 1 > "$out/$tag.log" 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-trace \
    -d "$out/${tag}_sqc" -o run --output-format csv -- python3 tools/quick_bench.py --spp 200 --reps 1 > "$out/${tag}_sqc.log" 2>&1 || true
done
