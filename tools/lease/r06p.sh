# r06p: the round-6 final kernel (RNG merge): GPU suite, smoke, bench, rocprof stats of the bench,
# the VALU-issue counters and the HBM request-size counters of the timed instance
export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "1000 r06p_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r06p_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r06p_bench.log python3 -u bench.py --steps 20 --warmup 5" \
 "500 r06p_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r06p_prof -o r06p -- python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --cpu-budget-mt 0" \
 "400 r06p_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r06p_pv" \
 "900 r06p_pmc_bytes.log bash tools/pmc_bytes.sh gpurun_out/r06p_pb python3 tools/quick_bench.py --spp 1000 --reps 1"
python3 tools/valu_summary.py gpurun_out/r06p_pv gpurun_out/r06p_valu.json > gpurun_out/r06p_valu_summary.log 2>&1
python3 tools/bytes_summary.py gpurun_out/r06p_pb rtp_render_pool > gpurun_out/r06p_bytes_summary.log 2>&1
