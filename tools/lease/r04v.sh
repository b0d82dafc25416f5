# r04v: two rays per lane in one instruction stream (lat_bench modes 11-13) against one ray (modes 0, 1)
bash tools/gpu_step.sh \
 "300 r04v_lat.log tools/lat_bench 2000 13 0 11 1 12"
