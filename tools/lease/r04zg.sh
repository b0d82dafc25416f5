# r04zg: the tile-deal edge cases (ranks without tiles) on hardware
bash tools/gpu_step.sh "300 r04zg_tiles.log python -u -m pytest tests/test_gpu_tiles.py -x -v --timeout 120 --timeout-method thread"
