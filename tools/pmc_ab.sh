#!/bin/bash
# One SQ pass (VALU, SALU, SMEM, waiting) of a 200-spp C2 render per librtp build; summarise with
# tools/pmc_summary.py gpurun_out/pmc_<name>.  usage: tools/pmc_ab.sh main build_exp/x.so ...
export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  if [ "$lib" = main ]; then unset RTP_LIB_PATH; else export RTP_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_$tag/p0 -o run --output-format csv -- python3 tools/quick_bench.py --spp 200 --reps 1 > gpurun_out/pmc_$tag.log 2>&1 || exit 1
done
