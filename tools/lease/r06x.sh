# r06x: C5's whole frame (3840x2160, 16384 spp, depth 50) on one MI355X with the final kernel
bash tools/gpu_step.sh \
 "400 r06x_c5_one_gpu.log python3 -u bench.py --workload c5 --steps 1 --warmup 0 --cpu-budget 0 --cpu-budget-mt 0"
