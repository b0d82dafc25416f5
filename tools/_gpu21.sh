bash tools/gpu_step.sh \
 "400 r04c_bvhtests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py -k 'c3 or bvh or sphere or lds' -x -v --timeout 300 --timeout-method thread" \
 "1000 r04c_ab_c3.log bash tools/ab_c3.sh 2 variants/base.so variants/p0.so main variants/p16.so variants/p48.so variants/p24.so"
