bash tools/gpu_step.sh \
 "300 r03q_c1.log python3 tools/quick_bench.py --nx 200 --ny 200 --spp 10 --depth 10 --reps 3" \
 "900 r03q_shares.log bash tools/share_sweep.sh '2 4 8' 'default'" \
 "400 r03q_valu.log bash tools/pmc_valu.sh gpurun_out/r03q_valu" \
 "900 r03q_bytes.log bash tools/pmc_bytes.sh gpurun_out/r03q_bytes python3 tools/quick_bench.py --tiles --spp 1000 --reps 1"
