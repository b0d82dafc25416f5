# r04y: C4's 1/8 share on whole tiles (1920x1088), the pixel-list instance (bench.py's path for 1080 rows)
# against the tile-deal instance (pixel coordinates computed in the kernel), same pixels, kernel ms
bash tools/gpu_step.sh \
 "300 r04y_list.log python3 tools/quick_bench.py --share --nx 1920 --ny 1088 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04y_tiles.log python3 tools/quick_bench.py --tiles --nx 1920 --ny 1088 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04y_list2.log python3 tools/quick_bench.py --share --nx 1920 --ny 1088 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04y_tiles2.log python3 tools/quick_bench.py --tiles --nx 1920 --ny 1088 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2"
