# r05l: clean timing bounds (same images): the rotated-box scan groups run twice
bash tools/gpu_step.sh \
 "900 r05l_ab_c2.log bash tools/ab.sh 2 main build_exp/lib_dup79.so build_exp/lib_dup100.so"
