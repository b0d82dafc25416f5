bash tools/gpu_step.sh \
 "300 r03c_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r03c_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r03c_dbg8.log python -u tools/dbg_stats.py --spp 1000 --world 8" \
 "300 r03c_dbg1.log python -u tools/dbg_stats.py --spp 1000" \
 "900 r03c_ab.log bash tools/ab_c2_tiles.sh 3 main variants/hist_slot.so variants/prex_lds.so variants/no_hist.so"
