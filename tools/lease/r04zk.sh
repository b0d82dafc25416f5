# r04zk: last check of the tree the round ends with: GPU suite, smoke, bench
bash tools/gpu_step.sh \
 "900 r04zk_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r04zk_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r04zk_bench.log python3 -u bench.py"
