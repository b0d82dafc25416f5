# r06l: the dielectric and Lambertian RNG draws taken in one pass (shade_hit):
# exactness (goldens incl. the C2 full frame, glass subsets, C3, stealing) and a same-box A/B
# against the previous kernel (build_exp/lib_base.so = HEAD before the change)
bash tools/gpu_step.sh \
 "500 r06l_tests.log python -u -m pytest tests/test_golden.py tests/test_gpu_steal.py tests/test_gpu_bvh.py -m gpu -x -v --timeout 300 --timeout-method thread" \
 "600 r06l_ab_c2.txt bash tools/ab.sh 3 main build_exp/lib_base.so" \
 "600 r06l_ab_c3.txt bash tools/ab_c3.sh 2 main build_exp/lib_base.so"
