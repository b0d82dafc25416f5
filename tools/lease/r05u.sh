# r05u: READY entries carrying their seed (one LDS round trip per refill) and the camera's sqrt through
# sqrt_exact: exactness (digests, golden/parity tests through the combined build) and A/B
bash tools/gpu_step.sh \
 "120 r05u_digest_base.log env RTP_LIB_PATH=build_exp/lib_m_base.so python3 tools/lib_digest.py --nx 800 --ny 800 --spp 64" \
 "120 r05u_digest_rscs.log env RTP_LIB_PATH=build_exp/lib_m_rscs.so python3 tools/lib_digest.py --nx 800 --ny 800 --spp 64" \
 "600 r05u_tests.log env RTP_LIB_PATH=build_exp/lib_m_rscs.so python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_steal.py tests/test_gpu_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "900 r05u_ab_c2.log bash tools/ab.sh 2 build_exp/lib_m_base.so build_exp/lib_m_rs.so build_exp/lib_m_cs.so build_exp/lib_m_rscs.so" \
 "900 r05u_ab_c4s8.log env QB_ARGS='--nx 1920 --ny 1080 --spp 4096 --tiles --world 8 --rank 0' bash tools/ab.sh 1 build_exp/lib_m_base.so build_exp/lib_m_rs.so build_exp/lib_m_rscs.so"
