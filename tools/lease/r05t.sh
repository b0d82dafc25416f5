# r05t: every BASELINE.json configuration on one GPU with the round-5 build
bash tools/gpu_step.sh "600 r05t_configs.log bash tools/configs_bench.sh gpurun_out/r05t_configs"
