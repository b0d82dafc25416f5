bash tools/gpu_step.sh \
 "900 r03b_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "300 r03b_bench.log python -u bench.py --steps 10 --warmup 2" \
 "240 r03b_setup_auto.log python -u tools/setup_cost.py --ff-tables auto" \
 "240 r03b_setup_on.log python -u tools/setup_cost.py --ff-tables on" \
 "300 r03b_plan1.log python -u tools/plan_experiment.py" \
 "300 r03b_plan2.log python -u tools/plan_experiment.py --world 2" \
 "300 r03b_plan8.log python -u tools/plan_experiment.py --world 8" \
 "300 r03b_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r03b_valu" \
 "600 r03b_ab_hist.log bash tools/ab_c2_tiles.sh 3 main variants/hist_slot.so variants/no_hist.so" \
 "600 r03b_share_sweep.log bash tools/share_sweep.sh '8 4' '64 32 16'"
