# r06y: bench.py's other modes on small frames after the round-6 changes (self-launch, tree sum,
# fixtures): N = 1 c4 / c5 / tile launch, N = 2 gloo rehearsals of the tile shard (c4) and of weak scaling
C="--steps 2 --warmup 1 --cpu-budget 0 --cpu-budget-mt 0 --ff-tables off"
bash tools/gpu_step.sh \
 "200 r06y_c4_n1.log python3 -u bench.py --workload c4 --nx 256 --ny 128 --spp 16 $C" \
 "200 r06y_c5_n1.log python3 -u bench.py --workload c5 --nx 96 --ny 64 --spp 64 $C" \
 "200 r06y_tiles_n1.log python3 -u bench.py --workload c2 --n1-launch tiles --nx 160 --ny 160 --spp 8 $C" \
 "300 r06y_c4_n2.log python3 -u bench.py --gpus 2 --dist-backend gloo --share-gpu --workload c4 --nx 128 --ny 64 --spp 8 --check $C" \
 "300 r06y_weak_n2.log python3 -u bench.py --gpus 2 --dist-backend gloo --share-gpu --scaling weak --workload c2 --nx 64 --ny 64 --spp 8 $C" \
 "300 r06y_c5_n3.log python3 -u bench.py --gpus 3 --dist-backend gloo --share-gpu --workload c5 --nx 96 --ny 64 --spp 96 --check $C"
