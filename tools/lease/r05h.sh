# r05h: timing bounds (wrong images): no exact scan of the rotated-box quads / no quad pdf / no sphere pdf
bash tools/gpu_step.sh \
 "900 r05h_ab_c2.log bash tools/ab.sh 2 main build_exp/lib_b_rot.so build_exp/lib_b_qpdf.so build_exp/lib_b_spdf.so" \
 "900 r05h_ab_c4s8.log env QB_ARGS='--nx 1920 --ny 1080 --spp 4096 --tiles --world 8 --rank 0' bash tools/ab.sh 1 main build_exp/lib_b_rot.so build_exp/lib_b_qpdf.so build_exp/lib_b_spdf.so"
