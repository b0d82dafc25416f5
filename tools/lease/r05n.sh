# r05n: the rotated boxes' vertical faces in the closest-hit prefilter (PreVert keys, three candidates,
# generic exact candidate test): exactness first, then A/B against HEAD and against RTP_PREFILTER_VERT=0
bash tools/gpu_step.sh \
 "600 r05n_tests.log python -u -m pytest tests/test_gpu_prefilter.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_steal.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "900 r05n_ab_c2.log bash tools/ab.sh 2 build_exp/lib_head.so main" \
 "900 r05n_ab_env_c2.log bash tools/ab_env.sh 1 - RTP_PREFILTER_VERT=0" \
 "900 r05n_ab_c4s8.log env QB_ARGS='--nx 1920 --ny 1080 --spp 4096 --tiles --world 8 --rank 0' bash tools/ab.sh 1 build_exp/lib_head.so main"
