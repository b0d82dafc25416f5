export TMPDIR=/tmp
# r04a: (1) uint32 cursors + stealing-aware priority lag vs HEAD (C2: no stealing; C4 at 1024 spp: stealing)
#       (2) C4 tile-deal shares; (3) the GPU tests incl. the new full-size / statistics / depth tests;
#       (4) refreshed C2 PMC (HBM bytes, VALU issue)
bash tools/gpu_step.sh \
 "400 r04a_ab_c2.log bash tools/ab.sh 2 main build_exp/head.so" \
 "600 r04a_ab_c4.log env QB_ARGS='--nx 1920 --ny 1080 --spp 1024' bash tools/ab.sh 2 main build_exp/head.so build_exp/prio0.so" \
 "600 r04a_c4_shares.log bash tools/c4_shares.sh" \
 "900 r04a_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "900 r04a_pmc_bytes.log bash tools/pmc_bytes.sh gpurun_out/r04a_pb python3 tools/quick_bench.py --tiles --spp 1000 --reps 1" \
 "300 r04a_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r04a_pv"
