# r04ze: history rows prefetched per light-hit sample in the fast-forward batch (kHistPrefetch 3 / 4 / 8 against 6)
bash tools/gpu_step.sh \
 "500 r04ze_ab_c2.log bash tools/ab.sh 2 main build_exp/pf3.so build_exp/pf4.so build_exp/pf8.so" \
 "500 r04ze_ab_c4s8.log env QB_ARGS='--tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0' bash tools/ab.sh 2 main build_exp/pf3.so build_exp/pf4.so build_exp/pf8.so"
