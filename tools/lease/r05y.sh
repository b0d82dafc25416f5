# r05y: bench.py's C5 frame on one GPU (whole frame, contiguous launch) with the stderr heartbeat; the C5 bench tests
bash tools/gpu_step.sh \
 "400 r05y_c5_n1.log python3 -u bench.py --workload c5 --steps 2 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "400 r05y_c5_tests.log python -u -m pytest tests/test_gpu_bench_c5.py tests/test_gpu_rccl.py -m gpu -v --timeout 300 --timeout-method thread"
