# r05d: instruction mix of the production pool kernel (C2, C2 1/8, C4 1/8)
bash tools/gpu_step.sh "600 r05d_pmc_pool.log bash tools/pmc_pool.sh gpurun_out/r05d_pool c2 c2s8 c4s8"
