# r04zi: C3's walk with the next node of a sphere leaf loaded before the leaf's exact test (build_exp/leafpf.so), bit-exactness by digest
bash tools/gpu_step.sh \
 "200 r04zi_digest_main.log python3 tools/lib_digest.py --variant 3 --nx 512 --ny 512 --spp 8" \
 "200 r04zi_digest_pf.log env RTP_LIB_PATH=build_exp/leafpf.so python3 tools/lib_digest.py --variant 3 --nx 512 --ny 512 --spp 8" \
 "500 r04zi_ab_c3.log bash tools/ab_c3.sh 3 main build_exp/leafpf.so"
