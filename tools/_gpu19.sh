bash tools/gpu_step.sh \
 "900 r03s_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 r03s_bench.log python -u bench.py --steps 10 --warmup 2" \
 "300 r03s_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s_prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0" \
 "400 r03s_valu.log bash tools/pmc_valu.sh gpurun_out/r03s_valu" \
 "900 r03s_bytes.log bash tools/pmc_bytes.sh gpurun_out/r03s_bytes python3 tools/quick_bench.py --tiles --spp 1000 --reps 1"
