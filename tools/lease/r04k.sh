export TMPDIR=/tmp
# r04k: Markstein roots for the sphere tests + the generator's cos_theta_max reused by the sphere pdf
#       (no recompute branch): fast-math device checks (kind 9), GPU tests, A/B vs HEAD (C2 N=1, C2 1/8 share, C3)
bash tools/gpu_step.sh \
 "300 r04k_fastmath.log python -u -m pytest tests/test_gpu_fast_math.py -x -v --timeout 240 --timeout-method thread" \
 "900 r04k_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "400 r04k_ab_c2.log bash tools/ab.sh 2 main build_exp/head.so" \
 "400 r04k_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/head.so" \
 "400 r04k_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/head.so"
