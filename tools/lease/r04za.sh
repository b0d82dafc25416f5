# r04za: C4 shares through the tile instance (bench.py's N > 1 path since r04z), N = 1, 2, 4, 8
bash tools/gpu_step.sh "900 r04za_c4_shares.log bash tools/c4_shares.sh"
