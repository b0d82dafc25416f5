export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "700 r03y_configs.log bash tools/configs_bench.sh gpurun_out/r03y_configs" \
 "200 r03y_pmc_ta.log rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU --kernel-trace -d gpurun_out/r03y/pmc_ta -o run --output-format csv -- python3 tools/quick_bench.py --nx 2048 --ny 2048 --spp 16 --variant 3 --reps 1"
