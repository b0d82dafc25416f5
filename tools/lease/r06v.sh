# r06v: the final round-6 tree: the whole GPU suite and smoke
bash tools/gpu_step.sh \
 "1000 r06v_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r06v_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'"
