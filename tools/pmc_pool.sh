#!/bin/bash
# Dynamic instruction mix of the production pool kernel (the instances bench.py
# and the shard ranks launch), two SQ counter passes per workload:
#   c2      C2 800x800x1000 spp, contiguous (bench.py's N = 1 instance)
#   c2s8    C2's 1/8 tile share (rank 0 of 8, tile instance)
#   c4s8    C4's 1/8 tile share (1920x1080x4096, rank 0 of 8, tile instance)
#   c5s8    C5's 1/8 sample share (3840x2160x2048 spp, contiguous, work stealing)
# tools/pool_pmc_summary.py prints per-launch totals and per live bounce.
# usage: tools/pmc_pool.sh <outdir> [workloads...]   (GPU box, repo root)
export TMPDIR=/tmp
out=$1; shift
wls=${*:-"c2 c2s8 c4s8"}
mkdir -p "$out"
for wl in $wls; do
  case $wl in
    c2) args="--spp 1000 --reps 1" ;;
    c2s8) args="--spp 1000 --reps 1 --tiles --world 8 --rank 0" ;;
    c4s8) args="--nx 1920 --ny 1080 --spp 4096 --reps 1 --tiles --world 8 --rank 0" ;;
    c5s8) args="--nx 3840 --ny 2160 --spp 2048 --reps 1" ;;
    *) echo "unknown workload $wl"; exit 1 ;;
  esac
  i=0; mkdir -p "$out/$wl"
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    echo "$wl pass $i"
    timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace -d "$out/$wl/p$i" -o run --output-format csv \
      -- python3 tools/quick_bench.py $args > "$out/$wl/p$i.log" 2>&1 || exit 1
  done
done
python3 tools/pool_pmc_summary.py "$out" $wls
