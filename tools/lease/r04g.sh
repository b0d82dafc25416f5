export TMPDIR=/tmp
# r04g: HEAD (pow5/Markstein) measured for the docs: configs C1-C5, C4 tile-deal shares 1/2/4/8,
#       stats (N=1, C2 1/8 share), VALU and HBM-byte counters of the bench kernel, rocprof stats of bench
bash tools/gpu_step.sh \
 "900 r04g_configs.log bash tools/configs_bench.sh gpurun_out/r04g_configs" \
 "900 r04g_c4_shares.log bash tools/c4_shares.sh" \
 "300 r04g_dbg1.log python3 tools/dbg_stats.py --spp 200" \
 "300 r04g_dbg8.log python3 tools/dbg_stats.py --spp 1000 --world 8" \
 "300 r04g_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r04g_pv" \
 "900 r04g_pmc_bytes.log bash tools/pmc_bytes.sh gpurun_out/r04g_pb python3 tools/quick_bench.py --tiles --spp 1000 --reps 1" \
 "400 r04g_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_prof -o bench --output-format csv -- python3 -u bench.py"
