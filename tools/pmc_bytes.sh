#!/bin/bash
# HBM request-size counter passes (one counter per rocprofv3 run, --kernel-trace only).
# Bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (reads, as classified by
# tools/bytes_summary.py) and 32/64 B write requests; checked against known byte
# counts with tools/calib_fetch.  Run on the GPU box from the repo root.
# usage: tools/pmc_bytes.sh <outdir> <program + args...>   (program: python3 script or binary)
export TMPDIR=/tmp
out=$1; shift
set -e
mkdir -p "$out"
i=0
for c in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM \
         TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WRREQ_DRAM FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$out/p$i" -o run --output-format csv -- "$@" > "$out/p$i.log" 2>&1
done
