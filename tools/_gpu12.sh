bash tools/gpu_step.sh \
 "600 r03l_wpx2.log env QB_ARGS='--tiles --spp 1000 --world 2 --rank 0' bash tools/ab_env.sh 2 RTP_WAVE_PIXELS=80 RTP_WAVE_PIXELS=96 RTP_WAVE_PIXELS=112" \
 "600 r03l_wpx4.log env QB_ARGS='--tiles --spp 1000 --world 4 --rank 0' bash tools/ab_env.sh 2 RTP_WAVE_PIXELS=80 RTP_WAVE_PIXELS=96 RTP_WAVE_PIXELS=112" \
 "600 r03l_wpx8.log env QB_ARGS='--tiles --spp 1000 --world 8 --rank 0' bash tools/ab_env.sh 2 - RTP_WAVE_PIXELS=72 RTP_WAVE_PIXELS=80" \
 "600 r03l_wpx3.log env QB_ARGS='--tiles --spp 1000 --world 3 --rank 0' bash tools/ab_env.sh 1 - RTP_WAVE_PIXELS=96"
