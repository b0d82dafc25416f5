# r05k: branch-free non-parallelogram quads (RTP_NONPARA_BF=1, in-tree) vs the branch (lib_np0): A/B + exactness
bash tools/gpu_step.sh \
 "900 r05k_ab_c2.log bash tools/ab.sh 2 build_exp/lib_np0.so main" \
 "900 r05k_ab_c4s8.log env QB_ARGS='--nx 1920 --ny 1080 --spp 4096 --tiles --world 8 --rank 0' bash tools/ab.sh 1 build_exp/lib_np0.so main" \
 "600 r05k_tests.log python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_prefilter.py tests/test_gpu_direct.py -m gpu -x -q --timeout 300 --timeout-method thread"
