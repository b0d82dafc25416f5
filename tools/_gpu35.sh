export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "900 r03z3_ab_drop.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab_env.sh 2 - RTP_BVH_DROP=1 RTP_BVH_DROP=3 RTP_BVH_DROP_SA=0.55 RTP_BVH_DROP_SA=0.65"
