# r06n: three small shading changes, each behind a macro: sphere normals as Markstein divisions
# (RTP_SPH_NORMAL_MK), the path end's LDS adds (RTP_LDS_ADD, non-walk instances), a quad hit's
# ONB w from the table (RTP_QUAD_W).  Exactness, then a same-box A/B of main (all three) against
# HEAD (lib_base: none) and each one switched off
bash tools/gpu_step.sh \
 "500 r06n_tests.log python -u -m pytest tests/test_golden.py tests/test_gpu_steal.py tests/test_gpu_bvh.py tests/test_gpu_prefilter.py -m gpu -x -v --timeout 300 --timeout-method thread" \
 "900 r06n_ab_c2.txt bash tools/ab.sh 3 main build_exp/lib_base.so build_exp/lib_now.so build_exp/lib_nomk.so build_exp/lib_noadd.so" \
 "700 r06n_ab_c3.txt bash tools/ab_c3.sh 2 main build_exp/lib_base.so build_exp/lib_now.so"
