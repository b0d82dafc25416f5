export TMPDIR=/tmp
# r04j: the bench kernel's instruction mix and wait cycles (two SQ counter passes, --kernel-trace only),
#       and the list of counters this rocprofv3 offers on gfx950
mkdir -p gpurun_out/r04j
bash tools/gpu_step.sh \
 "120 r04j_list.log rocprofv3 -L" \
 "200 r04j_mix.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES --kernel-trace -d gpurun_out/r04j/mix -o run --output-format csv -- python3 tools/quick_bench.py --tiles --spp 1000 --reps 1" \
 "200 r04j_wait.log rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace -d gpurun_out/r04j/wait -o run --output-format csv -- python3 tools/quick_bench.py --tiles --spp 1000 --reps 1"
