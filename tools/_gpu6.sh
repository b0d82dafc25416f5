bash tools/gpu_step.sh \
 "600 r03f_c3_walks.log bash tools/c3_walks.sh 32 variants/lds_threaded.so" \
 "300 r03f_pmc_c3_global.log env RTP_BVH_LDS=0 bash tools/pmc_quick.sh gpurun_out/r03f_pmc_c3_global --nx 2048 --ny 2048 --spp 16 --variant 3 --reps 1" \
 "300 r03f_pmc_c3_lds.log bash tools/pmc_quick.sh gpurun_out/r03f_pmc_c3_lds --nx 2048 --ny 2048 --spp 16 --variant 3 --reps 1" \
 "600 r03f_ab.log bash tools/ab_c2_tiles.sh 3 main variants/hist_pf4.so variants/hist_pf6.so variants/head.so"
