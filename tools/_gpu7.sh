bash tools/gpu_step.sh \
 "600 r03g_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 r03g_bench.log python -u bench.py --steps 10 --warmup 2" \
 "300 r03g_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03g_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r03g_dbg1.log python -u tools/dbg_stats.py --spp 1000" \
 "300 r03g_dbg8.log python -u tools/dbg_stats.py --spp 1000 --world 8" \
 "300 r03g_share.log bash tools/share_sweep.sh '2 4 8' '64'"
