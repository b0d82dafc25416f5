# r06o: a longer same-box A/B (8 interleaved rounds, best of 3 renders each) of the round-6
# shading changes on C2: the kernel before the RNG merge (lib_premerge, 1081b2e), the RNG
# merge (lib_base, 7cbbb6a), + Markstein normals + quad w + LDS adds (main), + without the
# LDS adds (lib_noadd)
bash tools/gpu_step.sh \
 "1100 r06o_ab_c2.txt bash tools/ab.sh 8 main build_exp/lib_base.so build_exp/lib_premerge.so build_exp/lib_noadd.so"
