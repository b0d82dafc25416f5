# r05zc: rank 3 of 8's C5 share over the canvas' first 1080 rows (4 147 200 px x 2048 spp) against the oracle's digests
bash tools/gpu_step.sh "600 r05zc_c5_band_digest.log python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread"
