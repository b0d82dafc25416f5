export TMPDIR=/tmp
# r04d: closest_hit decomposition (lat_bench modes 0/5/6/7, HBM gather 4) with and without the |det| fallback branch;
#       C4 shares with the 128-px planner; bench --workload c4 once; the RCCL world-size-1 test
bash tools/gpu_step.sh \
 "300 r04d_lat.log ./tools/lat_bench 2000 5 0 6 7 4" \
 "300 r04d_lat_nofb.log ./tools/lat_bench_nofb 2000 0 6 7" \
 "600 r04d_c4_shares.log bash tools/c4_shares.sh '4 8'" \
 "300 r04d_bench_c4.log python3 -u bench.py --workload c4 --steps 1 --warmup 0 --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r04d_rccl.log python3 -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 240 --timeout-method thread"
