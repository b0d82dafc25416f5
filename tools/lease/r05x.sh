# r05x: the whole C4 frame against the oracle's digests (contiguous stealing launch and tile instance)
bash tools/gpu_step.sh "600 r05x_c4_digest.log python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread"
