# r06j: how often a whole wave's bounce step has no lane whose closest hit is a
# rotated-box face (the most a wave-uniform box reject could skip)
bash tools/gpu_step.sh \
 "300 r06j_box_free_c2.txt python -u tools/dbg_stats.py --spp 16" \
 "300 r06j_box_free_c2_share8.txt python -u tools/dbg_stats.py --spp 16 --world 8 --rank 3"
