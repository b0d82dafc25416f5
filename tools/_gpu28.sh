bash tools/gpu_step.sh \
 "500 r03v_bvhtests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py tests/test_gpu_prefilter.py tests/test_golden.py -k 'c3 or bvh or sphere or lds or prefilter or glass' -x -v --timeout 300 --timeout-method thread" \
 "900 r03v_ab_c3.log bash tools/ab_c3.sh 2 main variants/nopair.so"
