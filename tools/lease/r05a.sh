# r05a: round-5 first box: GPU suite (incl. the C5 rehearsal), the default
# bench (C2 + scaling anchors), C5 rank shares on one GPU
bash tools/gpu_step.sh \
 "900 r05a_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "400 r05a_bench.log python3 -u bench.py" \
 "600 r05a_c5_shares.log bash tools/c5_shares.sh"
