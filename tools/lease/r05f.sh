# r05f: deferred sphere leaves with the record kept in registers (no re-read): exactness + A/B
bash tools/gpu_step.sh \
 "120 r05f_digest_d24r.log env RTP_LIB_PATH=build_exp/lib_d24r.so python3 tools/lib_digest.py --nx 512 --ny 512 --spp 8 --variant 3" \
 "600 r05f_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/lib_d8r.so build_exp/lib_d24r.so build_exp/lib_d48r.so"
