bash tools/gpu_step.sh \
 "600 r03d_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 r03d_bench.log python -u bench.py --steps 10 --warmup 2" \
 "600 r03d_ab.log bash tools/ab_c2_tiles.sh 3 main variants/hist_nostore.so variants/hist_noload.so" \
 "300 r03d_dbg_c3.log python -u tools/dbg_stats.py --spp 16 --n 2048 --variant 3" \
 "600 r03d_configs.log bash tools/configs_bench.sh gpurun_out/r03d_configs"
