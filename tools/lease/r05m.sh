# r05m: clean timing bounds (same images): kinds 7..8 scanned twice; the axis quads' prefilter keys twice
bash tools/gpu_step.sh \
 "900 r05m_ab_c2.log bash tools/ab.sh 2 main build_exp/lib_dup78.so build_exp/lib_duppre.so"
