bash tools/gpu_step.sh \
 "900 r03u_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200 r03u_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 r03u_bench.log python -u bench.py --steps 10 --warmup 2" \
 "600 r03u_configs.log bash tools/configs_bench.sh gpurun_out/r03u_configs"
