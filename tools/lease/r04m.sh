export TMPDIR=/tmp
# r04m: planned-render / two-context tests; C3 texture-path counters (L1 hit rate, L2 latency,
#       TD/TA stalls) of the global walk; non-temporal node gathers A/B (build_exp/bvhnt.so)
mkdir -p gpurun_out/r04m
bash tools/gpu_step.sh \
 "400 r04m_tests.log python -u -m pytest tests/test_gpu_planned_concurrency.py -x -v --timeout 300 --timeout-method thread" \
 "200 r04m_c3_tcp.log timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r04m/tcp -o run --output-format csv -- python3 tools/quick_bench.py --nx 2048 --ny 2048 --spp 16 --variant 3 --reps 1" \
 "400 r04m_ab_c3_nt.log bash tools/ab_c3.sh 2 main build_exp/bvhnt.so"
