bash tools/gpu_step.sh \
 "900 r03x_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200 r03x_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 r03x_bench.log python -u bench.py --steps 10 --warmup 2" \
 "300 r03x_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03x_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "700 r03x_ab_walk.log env QB_ARGS='--nx 2048 --ny 2048 --spp 16 --variant 3' bash tools/ab.sh 2 main variants/walk40.so variants/walk56.so"
