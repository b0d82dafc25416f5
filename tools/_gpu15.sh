bash tools/gpu_step.sh \
 "600 r03o_balance.log python -u tools/balance_plan.py" \
 "600 r03o_c3bins.log bash tools/ab_c3.sh 2 main variants/bins64.so"
