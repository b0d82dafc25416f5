export TMPDIR=/tmp
# r04b: exec occupancy per region (stats build) at N = 1 and the C2 1/8 share; C4 share px/wave sweep;
#       C2 A/B of the stats-instrumented tree against r04a (production code must be unchanged)
bash tools/gpu_step.sh \
 "300 r04b_ab_c2.log bash tools/ab.sh 2 main build_exp/r04a.so" \
 "300 r04b_dbg1.log python3 tools/dbg_stats.py --spp 200" \
 "300 r04b_dbg8.log python3 tools/dbg_stats.py --spp 1000 --world 8" \
 "900 r04b_c4_px.log env QB_ARGS='--share --nx 1920 --ny 1080 --spp 4096' bash tools/share_sweep.sh '8 4' 'default 64 96 128'"
