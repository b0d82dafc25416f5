# r05zd: rank 3 of 8's whole C5 share (3840x2160 x 2048 spp, 1.7e10 samples) against the oracle's digests
bash tools/gpu_step.sh "600 r05zd_c5_full_digest.log python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread"
