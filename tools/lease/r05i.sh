# r05i: finer timing bounds: skip kinds 7..9 / skip kinds 10 and 0 (wrong images); the scene's quad groups
RTP_VERBOSE=1 timeout -k 10 120 python3 tools/quick_bench.py --spp 1 --reps 1 2>&1 | grep "rtp:" > gpurun_out/r05i_groups.log
bash tools/gpu_step.sh \
 "900 r05i_ab_c2.log bash tools/ab.sh 2 build_exp/lib_b_main2.so build_exp/lib_b_rot.so build_exp/lib_b_rot79.so build_exp/lib_b_rot100.so"
