export TMPDIR=/tmp
# r04l: one table read per lane per fast-forward batch (RTP_FF_STEP=1, build_exp/ffstep.so) against HEAD:
#       correctness (golden C2 frame, stealing, full-size C3/C4/C5) on the variant, then A/B C2 N=1, C2 1/8, C4 1/8
bash tools/gpu_step.sh \
 "600 r04l_tests_ffstep.log env RTP_LIB_PATH=build_exp/ffstep.so python -u -m pytest tests/test_golden.py tests/test_gpu_steal.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread" \
 "400 r04l_ab_c2.log bash tools/ab.sh 2 main build_exp/head.so build_exp/ffstep.so" \
 "400 r04l_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/head.so build_exp/ffstep.so" \
 "600 r04l_ab_c4_s8.log env QB_ARGS='--share --nx 1920 --ny 1080 --spp 4096 --world 8 --rank 0' bash tools/ab.sh 2 main build_exp/head.so build_exp/ffstep.so"
