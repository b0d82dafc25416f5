# r04zj: the pair-node walk (build_exp/pair.so, RTP_BVH_PAIR=1): digests against main on C3's scene,
# the BVH parity tests through it, then C3 timing A/B
bash tools/gpu_step.sh \
 "200 r04zj_digest_main.log python3 tools/lib_digest.py --variant 3 --nx 512 --ny 512 --spp 8" \
 "200 r04zj_digest_pair.log env RTP_LIB_PATH=build_exp/pair.so python3 tools/lib_digest.py --variant 3 --nx 512 --ny 512 --spp 8" \
 "400 r04zj_tests_pair.log env RTP_LIB_PATH=build_exp/pair.so python -u -m pytest tests/test_gpu_bvh.py tests/test_golden.py -x -v --timeout 200 --timeout-method thread" \
 "500 r04zj_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/pair.so"
