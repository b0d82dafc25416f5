export TMPDIR=/tmp
# r04n: (1) the SLP vectorizer off (build_exp/noslp.so: fewer packed-FP32 ops and s_nop hazards) A/B on C2, its 1/8
#       share and C3; (2) the LDS-walk ceiling on C3's first 300 spheres: global walk vs LDS walk with one-sphere
#       leaves (build_exp/ldsleaf1.so) vs the leaves-of-6 LDS walk; (3) fewer distinct octant copies for the
#       global walk (RTP_BVH_OCT_MASK 7 = 8 copies, 5 = 4, 1 = 2, 0 = 1)
bash tools/gpu_step.sh \
 "400 r04n_ab_c2.log bash tools/ab.sh 2 main build_exp/noslp.so" \
 "400 r04n_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/noslp.so" \
 "400 r04n_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/noslp.so" \
 "200 r04n_ceil_global.log env RTP_BVH_LDS=0 python3 tools/c3_lds_ceiling.py" \
 "200 r04n_ceil_lds1.log env RTP_BVH_LDS=1 RTP_LIB_PATH=build_exp/ldsleaf1.so python3 tools/c3_lds_ceiling.py" \
 "200 r04n_ceil_lds6.log env RTP_BVH_LDS=1 python3 tools/c3_lds_ceiling.py" \
 "600 r04n_ab_c3_octmask.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 RTP_BVH_OCT_MASK=7 RTP_BVH_OCT_MASK=5 RTP_BVH_OCT_MASK=1 RTP_BVH_OCT_MASK=0"
