bash tools/gpu_step.sh \
 "300 r03k_chain1.log python -u tools/chain_floor.py" \
 "300 r03k_chain8.log python -u tools/chain_floor.py --world 8" \
 "300 r03k_chain2.log python -u tools/chain_floor.py --world 2" \
 "300 r03k_setup.log python -u tools/setup_cost.py --ff-tables auto --renders 2" \
 "600 r03k_wpx2.log env QB_ARGS='--tiles --spp 1000 --world 2 --rank 0' bash tools/ab_env.sh 2 - RTP_WAVE_PIXELS=96 RTP_WAVE_PIXELS=128" \
 "600 r03k_wpx4.log env QB_ARGS='--tiles --spp 1000 --world 4 --rank 0' bash tools/ab_env.sh 2 - RTP_WAVE_PIXELS=96 RTP_WAVE_PIXELS=128" \
 "600 r03k_wpx8.log env QB_ARGS='--tiles --spp 1000 --world 8 --rank 0' bash tools/ab_env.sh 2 - RTP_WAVE_PIXELS=96 RTP_WAVE_PIXELS=128"
