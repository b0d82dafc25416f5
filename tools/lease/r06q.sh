# r06q: the fixed-association tree reduce: the multi-rank C5 rehearsals and the one-rank RCCL path
# (gloo / nccl), then a probe of the tree over RCCL with 2 and 4 ranks sharing the GPU (RCCL may
# refuse duplicate devices: then the probe reports that and nothing else runs after it)
bash tools/gpu_step.sh \
 "600 r06q_tests.log python -u -m pytest tests/test_gpu_bench_c5.py tests/test_gpu_rccl.py tests/test_shard.py -v --timeout 300 --timeout-method thread" \
 "120 r06q_probe2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29671 tools/rccl_tree_probe.py" \
 "120 r06q_probe4.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29673 tools/rccl_tree_probe.py"
