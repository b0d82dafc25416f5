bash tools/gpu_step.sh \
 "300 r04g_fastmath.log python -u -m pytest tests/test_gpu_fast_math.py -x -q --timeout 250 --timeout-method thread" \
 "500 r04g_bvhtests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py tests/test_gpu_prefilter.py tests/test_golden.py -k 'c3 or bvh or sphere or lds or prefilter or glass' -x -v --timeout 300 --timeout-method thread" \
 "900 r04g_ab_c3.log bash tools/ab_c3.sh 2 variants/cw.so main variants/nofma.so variants/nodiv.so"
