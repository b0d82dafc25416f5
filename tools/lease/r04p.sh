export TMPDIR=/tmp
# r04p: compiler-option sweep on the no-SLP tree: -O2, -fno-unroll-loops, max-ilp and iterative-minreg scheduling;
#       C2 contiguous, C2 tile instance (the bench's), C3
bash tools/gpu_step.sh \
 "500 r04p_ab_c2.log bash tools/ab.sh 2 main build_exp/o2.so build_exp/nounroll.so build_exp/maxilp.so build_exp/minreg.so" \
 "500 r04p_ab_c2_tiles.log env QB_ARGS='--tiles --spp 1000' bash tools/ab.sh 2 main build_exp/o2.so build_exp/nounroll.so build_exp/maxilp.so build_exp/minreg.so" \
 "500 r04p_ab_c3.log bash tools/ab_c3.sh 2 main build_exp/o2.so build_exp/nounroll.so build_exp/maxilp.so build_exp/minreg.so"
