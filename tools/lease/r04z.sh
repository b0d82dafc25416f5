# r04z: the tile instance on clipped canvases (C4's 1080 rows): GPU tests, a 2-rank gloo rehearsal of
# bench.py's N > 1 path on one GPU (--check: the reduced canvas equals a one-process render), and the
# C4 1/8 share's kernel time through bench's own path at N = 1 (tile instance, rank 0 of 8 emulated by quick_bench)
bash tools/gpu_step.sh \
 "600 r04z_tests.log python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_fullsize.py tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread" \
 "400 r04z_bench_rehearsal.log python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29671 bench.py --gpus 2 --share-gpu --dist-backend gloo --ff-tables off --workload c4 --spp 16 --steps 2 --warmup 1 --check --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r04z_s8_tiles.log python3 tools/quick_bench.py --tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04z_s8_list.log python3 tools/quick_bench.py --share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2"
