bash tools/gpu_step.sh \
 "300 r03h_tiles_test.log python -u -m pytest tests/test_gpu_tiles.py -x -v --timeout 240 --timeout-method thread -m gpu" \
 "600 r03h_ab.log bash tools/ab_c2_tiles.sh 3 main variants/noff.so variants/head.so" \
 "600 r03h_rehearsal_n2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --share-gpu --dist-backend gloo --ff-tables off --steps 2 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0 --check"
