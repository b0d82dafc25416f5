# r05e: C3 deferred sphere leaves (RTP_BVH_DEFER): bit-exactness (digests, BVH/golden/steal tests) and A/B
bash tools/gpu_step.sh \
 "120 r05e_digest_main.log python3 tools/lib_digest.py --nx 512 --ny 512 --spp 8 --variant 3" \
 "120 r05e_digest_d24.log env RTP_LIB_PATH=build_exp/lib_d24.so python3 tools/lib_digest.py --nx 512 --ny 512 --spp 8 --variant 3" \
 "120 r05e_digest_d24q1.log env RTP_LIB_PATH=build_exp/lib_d24q1.so python3 tools/lib_digest.py --nx 512 --ny 512 --spp 8 --variant 3" \
 "400 r05e_tests_d24.log env RTP_LIB_PATH=build_exp/lib_d24.so python -u -m pytest tests/test_gpu_bvh.py tests/test_golden.py tests/test_gpu_steal.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "900 r05e_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/lib_d16.so build_exp/lib_d24.so build_exp/lib_d32.so build_exp/lib_d24q1.so"
