# r06u: C3 at its full 256 spp over the canvas's first 128 rows (262 144 px) and its whole canvas
# at 16 spp, against the oracle's digests
bash tools/gpu_step.sh \
 "400 r06u_c3_digests.log python -u -m pytest tests/test_gpu_fullsize.py -k c3_whole -m gpu -v --timeout 300 --timeout-method thread"
