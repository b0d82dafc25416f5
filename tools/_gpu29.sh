bash tools/gpu_step.sh \
 "600 r03w_tests.log python -u -m pytest tests/test_gpu_steal.py tests/test_golden.py -x -v --timeout 300 --timeout-method thread" \
 "700 r03w_ab_c3.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 RTP_STEAL=1 RTP_STEAL=0" \
 "700 r03w_ab_c4.log env QB_ARGS='--nx 1920 --ny 1080 --spp 256' bash tools/ab_env.sh 2 RTP_STEAL=1 RTP_STEAL=0" \
 "700 r03w_ab_c5.log env QB_ARGS='--nx 3840 --ny 2160 --spp 64' bash tools/ab_env.sh 2 RTP_STEAL=1 RTP_STEAL=0"
