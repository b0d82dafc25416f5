# r05w: the scheduler's occupancy bias (100) and early if-conversion: more rounds, C4's 1/8 share, C3, exactness
bash tools/gpu_step.sh \
 "120 r05w_digest_base.log env RTP_LIB_PATH=build_exp/lib_m_base.so python3 tools/lib_digest.py --nx 800 --ny 800 --spp 64" \
 "120 r05w_digest_b100.log env RTP_LIB_PATH=build_exp/lib_f_b100ifc.so python3 tools/lib_digest.py --nx 800 --ny 800 --spp 64" \
 "1200 r05w_ab_c2.log bash tools/ab.sh 3 build_exp/lib_m_base.so build_exp/lib_f_bias100.so build_exp/lib_f_b100ifc.so" \
 "900 r05w_ab_c4s8.log env QB_ARGS='--nx 1920 --ny 1080 --spp 4096 --tiles --world 8 --rank 0' bash tools/ab.sh 1 build_exp/lib_m_base.so build_exp/lib_f_bias100.so build_exp/lib_f_b100ifc.so" \
 "900 r05w_ab_c3.log bash tools/ab_c3.sh 1 build_exp/lib_m_base.so build_exp/lib_f_bias100.so build_exp/lib_f_b100ifc.so"
