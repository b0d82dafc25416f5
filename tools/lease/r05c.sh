# r05c: per-step dynamic instruction counts of the bounce parts (tools/pmc_lat.sh on tools/lat_bench)
bash tools/gpu_step.sh "300 r05c_pmc_lat.log bash tools/pmc_lat.sh gpurun_out/r05c_lat 2000 5 0 6 7 3 1"
