bash tools/gpu_step.sh \
 "400 r04a_bvhtests.log python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py -k 'c3 or bvh or sphere or lds' -x -v --timeout 300 --timeout-method thread" \
 "900 r04a_ab_c3.log bash tools/ab_c3.sh 2 variants/base.so main variants/walk16.so variants/walk48.so variants/walk64.so"
