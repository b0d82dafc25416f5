set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 tools/ab_env.sh 2 "-" "RTP_BOXCULL=0" > gpurun_out/r06g_ab_env.txt 2>&1 || exit 1
timeout -k 10 600 tools/ab.sh 2 main build_exp/lib_base.so build_exp/lib_slim.so > gpurun_out/r06g_ab_libs.txt 2>&1 || exit 1
RTP_DEBUG_STATS=1 RTP_LIB_PATH=build_exp/lib_slim.so timeout -k 10 120 python tools/box_cull_rate.py --spp 16 > gpurun_out/r06g_slim_rates.txt 2>&1
