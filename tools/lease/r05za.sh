# r05za: the AUTO policy's direct stage from the measured chain allocation (rtp_host.cpp ff_auto_samples): its tests,
# the jump-table tests
bash tools/gpu_step.sh \
 "400 r05za_ff_tests.log python -u -m pytest tests/test_a_ff_policy.py tests/test_gpu_ff_tables.py -m gpu -v --timeout 300 --timeout-method thread"
