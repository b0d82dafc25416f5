bash tools/gpu_step.sh \
 "300 r03e_bvhtests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_golden.py -x -v --timeout 240 --timeout-method thread -m gpu" \
 "600 r03e_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 r03e_c3_lds.log python -u tools/quick_bench.py --nx 2048 --ny 2048 --spp 256 --variant 3 --reps 1" \
 "300 r03e_c3_global.log env RTP_BVH_LDS=0 python -u tools/quick_bench.py --nx 2048 --ny 2048 --spp 256 --variant 3 --reps 1" \
 "600 r03e_ab.log bash tools/ab_c2_tiles.sh 3 main variants/head.so"
