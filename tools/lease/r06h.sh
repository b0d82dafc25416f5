# r06h: the round-6 tree after the box-cull revert: GPU suite, smoke, bench, rocprof stats of the bench
bash tools/gpu_step.sh \
 "1000 r06h_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r06h_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r06h_bench.log python3 -u bench.py --steps 20 --warmup 5" \
 "500 r06h_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r06h_prof -o r06h -- python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --cpu-budget-mt 0"
