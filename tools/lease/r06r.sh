# r06r: C3's whole canvas (2048^2 x 16 spp, 1000 spheres) against the oracle's digests; every
# BASELINE.json configuration's kernel time on the final kernel (tools/configs_bench.sh)
bash tools/gpu_step.sh \
 "400 r06r_c3_digest.log python -u -m pytest tests/test_gpu_fullsize.py -k c3_whole -m gpu -v --timeout 300 --timeout-method thread" \
 "600 r06r_configs.log bash tools/configs_bench.sh gpurun_out/r06r_configs"
