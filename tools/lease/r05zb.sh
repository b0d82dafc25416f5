# r05zb: the tree with the adaptive AUTO policy and the bench heartbeat: GPU suite, smoke, bench
bash tools/gpu_step.sh \
 "900 r05zb_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r05zb_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r05zb_bench.log python3 -u bench.py --steps 20 --warmup 5"
