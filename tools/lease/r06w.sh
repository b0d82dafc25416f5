# r06w: 6 waves per SIMD again, now that the final kernel needs 81 VGPRs (80-VGPR cap: 2 dwords
# spilled in the contiguous instance, none in the tile instance): same-box A/B against main
bash tools/gpu_step.sh \
 "700 r06w_ab_c2.txt bash tools/ab.sh 6 main build_exp/lib_w6.so" \
 "500 r06w_ab_c2_tiles.txt env QB_ARGS='--spp 1000 --tiles' bash tools/ab.sh 4 main build_exp/lib_w6.so"
