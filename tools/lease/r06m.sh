# r06m: sphere hit normals as Markstein divisions by RN(1/r) (RTP_SPH_NORMAL_MK) and the path end's
# LDS adds without return (RTP_LDS_ADD): exactness, then a same-box A/B of main (both) against
# HEAD 7cbbb6a (lib_base: neither), lib_nomk (adds only), lib_noadd (Markstein only)
bash tools/gpu_step.sh \
 "500 r06m_tests.log python -u -m pytest tests/test_golden.py tests/test_gpu_steal.py tests/test_gpu_bvh.py -m gpu -x -v --timeout 300 --timeout-method thread" \
 "700 r06m_ab_c2.txt bash tools/ab.sh 3 main build_exp/lib_base.so build_exp/lib_nomk.so build_exp/lib_noadd.so" \
 "700 r06m_ab_c3.txt bash tools/ab_c3.sh 2 main build_exp/lib_base.so build_exp/lib_nomk.so"
