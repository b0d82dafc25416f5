export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "900 r03z2_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200 r03z2_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 r03z2_bench.log python -u bench.py --steps 10 --warmup 2" \
 "700 r03z2_configs.log bash tools/configs_bench.sh gpurun_out/r03z2_configs" \
 "300 r03z2_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03z2_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0"
