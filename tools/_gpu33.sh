export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "300 r03z_bvh_tests.log python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 200 --timeout-method thread" \
 "300 r03z_bvh_tests_drop3.log env RTP_BVH_DROP=3 RTP_BVH_DROP_SA=0.6 python -u -m pytest tests/test_golden.py tests/test_gpu_steal.py -x -q --timeout 120 --timeout-method thread" \
 "900 r03z_ab_drop.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 - RTP_BVH_DROP=1 RTP_BVH_DROP=2 RTP_BVH_DROP=3 RTP_BVH_DROP=4 RTP_BVH_DROP=5" \
 "900 r03z_ab_drop_sa.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 RTP_BVH_DROP=2 'RTP_BVH_DROP=2 RTP_BVH_DROP_SA=0.5' 'RTP_BVH_DROP=2 RTP_BVH_DROP_SA=0.6' 'RTP_BVH_DROP=2 RTP_BVH_DROP_SA=0.7' 'RTP_BVH_DROP=2 RTP_BVH_DROP_SA=0.8'" \
 "700 r03y_configs.log bash tools/configs_bench.sh gpurun_out/r03y_configs" \
 "200 r03y_pmc_ta.log rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU --kernel-trace -d gpurun_out/r03y/pmc_ta -o run --output-format csv -- python3 tools/quick_bench.py --nx 2048 --ny 2048 --spp 16 --variant 3 --reps 1"
