# r05z: the jump-table policy's costs on the round-5 build, fresh process each: no tables, the chain tables only
# (AUTO with the direct stage out of reach), all tables (tools/setup_cost.py: setup, first render, steady state)
bash tools/gpu_step.sh \
 "300 r05z_ff_off.log python3 tools/setup_cost.py --ff-tables off --renders 4" \
 "300 r05z_ff_chain.log env RTP_FF_AUTO_SAMPLES=1,999999999999999 python3 tools/setup_cost.py --ff-tables auto --renders 4" \
 "300 r05z_ff_on.log python3 tools/setup_cost.py --ff-tables on --renders 4"
