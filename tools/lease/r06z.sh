# r06z: the 8-rank C5 rehearsal at full size on one GPU through the round-6 path: bench.py --gpus 8
# started without a launcher (self-launch), gloo, shared device, tables off; the reduced frame
# (the fixed-association tree sum) against the oracle's N = 8 reduced-frame fixture
bash tools/gpu_step.sh \
 "1000 r06z_c5_rehearsal8.log python3 -u bench.py --gpus 8 --share-gpu --dist-backend gloo --workload c5 --steps 1 --warmup 0 --ff-tables off --cpu-budget 0 --cpu-budget-mt 0"
