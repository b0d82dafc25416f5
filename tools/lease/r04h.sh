export TMPDIR=/tmp
# r04h: the LDS-resident threaded sphere walk (leaves <= 6, 8 octant copies in each 16-wave block's LDS):
#       BVH / stealing / golden GPU tests, then C3 A/B against the global walk, then full C3
bash tools/gpu_step.sh \
 "600 r04h_bvh_tests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_steal.py -x -v --timeout 300 --timeout-method thread" \
 "900 r04h_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "600 r04h_ab_c3.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 - RTP_BVH_LDS=0" \
 "300 r04h_c3.log python3 tools/quick_bench.py --nx 2048 --ny 2048 --spp 256 --depth 50 --variant 3 --reps 1"
