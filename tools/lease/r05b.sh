# r05b: GPU suite; 8-rank C5 rehearsal on one GPU (gloo, shared device, tables off): the
# rank-3 shard against the c5_shard3_2048spp fixture and the t-test at full size
bash tools/gpu_step.sh \
 "900 r05b_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r05b_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "900 r05b_c5_rehearsal8.log python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29677 bench.py --gpus 8 --share-gpu --dist-backend gloo --workload c5 --steps 1 --warmup 0 --ff-tables off"
