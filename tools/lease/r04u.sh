export TMPDIR=/tmp
# r04u: the tree as committed (no-SLP build, contiguous bench launch): GPU tests, smoke, bench (defaults),
#       rocprof stats of bench, configs, C4 shares
bash tools/gpu_step.sh \
 "900 r04u_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r04u_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r04u_bench.log python3 -u bench.py" \
 "400 r04u_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04u_prof -o bench --output-format csv -- python3 -u bench.py" \
 "900 r04u_configs.log bash tools/configs_bench.sh gpurun_out/r04u_configs" \
 "900 r04u_c4_shares.log bash tools/c4_shares.sh"
