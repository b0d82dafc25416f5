# r05s: per-wave lifetimes of the C2 frame (how much of the launch its waves' tails leave idle)
bash tools/gpu_step.sh "300 r05s_wave_times.log python3 tools/wave_times.py --spp 1000"
