bash tools/gpu_step.sh \
 "300 r03q_c1.log python3 tools/quick_bench.py --nx 200 --ny 200 --spp 10 --depth 10 --reps 3" \
 "600 r03q_shares.log bash tools/share_sweep.sh '2 4 8' 'default'" \
 "300 r03r_parity.log env RTP_LIB_PATH=variants/chunk6.so python -u -m pytest tests/test_golden.py -x -q --timeout 240 --timeout-method thread -m gpu" \
 "900 r03r_ab1.log bash tools/ab_c2_tiles.sh 3 main variants/chunk6.so variants/chunk4.so" \
 "600 r03r_ab8.log bash tools/ab_share.sh 8 2 main variants/chunk6.so variants/chunk4.so" \
 "400 r03q_valu.log bash tools/pmc_valu.sh gpurun_out/r03q_valu" \
 "900 r03q_bytes.log bash tools/pmc_bytes.sh gpurun_out/r03q_bytes python3 tools/quick_bench.py --tiles --spp 1000 --reps 1"
