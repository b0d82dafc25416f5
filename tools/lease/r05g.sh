# r05g: the tree after the C3 experiment's removal: GPU suite (incl. the one-rank RCCL C5 path), smoke, bench
bash tools/gpu_step.sh \
 "900 r05g_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r05g_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r05g_bench.log python3 -u bench.py --steps 20 --warmup 5"
