# r05q: 6 waves per SIMD (80 VGPRs) with fewer history rows prefetched (one cold spill) vs 5 waves
RTP_VERBOSE=1 RTP_LIB_PATH=build_exp/lib_o6p4.so timeout -k 10 120 python3 tools/quick_bench.py --spp 1 --reps 1 2>&1 | grep "rtp:" > gpurun_out/r05q_occ.log
bash tools/gpu_step.sh \
 "900 r05q_ab_c2.log bash tools/ab.sh 2 main build_exp/lib_o6p4.so build_exp/lib_o6p6.so build_exp/lib_o5p4.so" \
 "900 r05q_ab_c2s8.log env QB_ARGS='--spp 1000 --tiles --world 8 --rank 0' bash tools/ab.sh 1 main build_exp/lib_o6p4.so build_exp/lib_o5p4.so"
