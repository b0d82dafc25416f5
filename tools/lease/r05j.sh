# r05j: the quads' 1/det without its |det| > 2^40 ballot branch (timing; same images on C2); quad groups
RTP_VERBOSE=1 timeout -k 10 120 python3 tools/quick_bench.py --spp 1 --reps 1 2>&1 | grep "rtp:" > gpurun_out/r05j_groups.log
bash tools/gpu_step.sh \
 "900 r05j_ab_c2.log bash tools/ab.sh 2 build_exp/lib_b_main2.so build_exp/lib_detfb0.so"
