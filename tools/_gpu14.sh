bash tools/gpu_step.sh \
 "900 r03n_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
 "900 r03n_shares.log bash tools/share_sweep.sh '1 2 3 4 8' '64 80'"
