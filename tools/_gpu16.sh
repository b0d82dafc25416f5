bash tools/gpu_step.sh \
 "900 r03p_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 r03p_bench.log python -u bench.py --steps 10 --warmup 2" \
 "300 r03p_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "600 r03p_configs.log bash tools/configs_bench.sh" \
 "600 r03p_rehearsal_n2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --share-gpu --dist-backend gloo --ff-tables off --steps 2 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0 --check"
