# r05ze: final tree of round 5: GPU suite (incl. the whole C5 share digest), smoke, bench
bash tools/gpu_step.sh \
 "900 r05ze_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r05ze_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r05ze_bench.log python3 -u bench.py --steps 20 --warmup 5"
