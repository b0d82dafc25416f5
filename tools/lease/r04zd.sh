# r04zd: bound of the fast-forward batch's history loads (build_exp/nohl.so: rows replaced by constants -- wrong images, timing only)
bash tools/gpu_step.sh \
 "400 r04zd_ab_c4s8.log env QB_ARGS='--tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0' bash tools/ab.sh 2 main build_exp/nohl.so" \
 "400 r04zd_ab_c2.log bash tools/ab.sh 2 main build_exp/nohl.so"
