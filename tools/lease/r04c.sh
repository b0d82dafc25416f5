export TMPDIR=/tmp
# r04c: latency microbenchmarks of the bounce parts (tools/lat_bench.hip), stats with dielectric/light counters,
#       px/wave sweeps of the C2 and C4 shares on the current kernel
bash tools/gpu_step.sh \
 "300 r04c_lat.log ./tools/lat_bench 2000 0 1 2 3 4" \
 "300 r04c_dbg1.log python3 tools/dbg_stats.py --spp 200" \
 "300 r04c_dbg8.log python3 tools/dbg_stats.py --spp 1000 --world 8" \
 "600 r04c_c2_px.log bash tools/share_sweep.sh '2 4 8' '64 80 96 112 128'" \
 "600 r04c_c4_px.log env QB_ARGS='--share --nx 1920 --ny 1080 --spp 4096' bash tools/share_sweep.sh '4 8' '80 96 112 128'"
