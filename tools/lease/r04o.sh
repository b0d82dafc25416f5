export TMPDIR=/tmp
# r04o: the tree built with -fno-slp-vectorize: GPU tests (bit-exactness), smoke, bench, rocprof stats, configs,
#       C4 shares; same-box A/B against the SLP build of the previous commit (build_exp/head.so)
bash tools/gpu_step.sh \
 "900 r04o_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r04o_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r04o_ab_c2.log bash tools/ab.sh 2 main build_exp/head.so" \
 "400 r04o_bench.log python3 -u bench.py" \
 "400 r04o_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof -o bench --output-format csv -- python3 -u bench.py --cpu-budget 0 --cpu-budget-mt 0" \
 "900 r04o_configs.log bash tools/configs_bench.sh gpurun_out/r04o_configs" \
 "900 r04o_c4_shares.log bash tools/c4_shares.sh"
