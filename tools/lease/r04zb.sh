# r04zb: final check at HEAD: the whole GPU suite, smoke, bench (N = 1 defaults)
bash tools/gpu_step.sh \
 "900 r04zb_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r04zb_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r04zb_bench.log python3 -u bench.py"
