export TMPDIR=/tmp
# r04r: 6 waves per SIMD (build_exp/occ6.so: 80 VGPRs, 4 dwords spilled in the C2 instances) vs 5 (main)
bash tools/gpu_step.sh \
 "400 r04r_ab_c2.log bash tools/ab.sh 2 main build_exp/occ6.so" \
 "400 r04r_ab_c2_tiles.log env QB_ARGS='--tiles --spp 1000' bash tools/ab.sh 2 main build_exp/occ6.so" \
 "400 r04r_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/occ6.so"
