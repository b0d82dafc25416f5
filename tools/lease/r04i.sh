export TMPDIR=/tmp
# r04i: (1) the split-intersection experiment in tools/lat_bench (modes 8/9 vs 0/1 at 1..5 waves per SIMD;
#       mode 10 checks the split hit against closest_hit); (2) C3 16 spp: global walk with leaves <= 6
#       (build_exp/leaf6.so, RTP_BVH_LDS=0) against the LDS walk and the leaf-1 global walk
bash tools/gpu_step.sh \
 "300 r04i_lat.log ./tools/lat_bench 2000 10 0 8 1 9" \
 "600 r04i_ab_c3_leaf.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 - RTP_BVH_LDS=0 'RTP_BVH_LDS=0 RTP_LIB_PATH=build_exp/leaf6.so'"
