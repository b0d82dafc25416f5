# r04x: C3 knobs re-checked on the final build: resumable-walk threshold (RTP_WALK_DONE 32/40/48/56)
# and dropped top boxes (RTP_BVH_DROP / RTP_BVH_DROP_SA env), C3 geometry at 16 spp
bash tools/gpu_step.sh \
 "500 r04x_ab_c3_walkdone.log bash tools/ab_c3.sh 2 main build_exp/wd32.so build_exp/wd40.so build_exp/wd56.so" \
 "300 r04x_c3_drop3.log env RTP_BVH_DROP=3 bash tools/ab_c3.sh 2 main" \
 "300 r04x_c3_sa05.log env RTP_BVH_DROP_SA=0.5 bash tools/ab_c3.sh 2 main" \
 "300 r04x_c3_sa07.log env RTP_BVH_DROP_SA=0.7 bash tools/ab_c3.sh 2 main"
