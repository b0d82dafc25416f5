export TMPDIR=/tmp
# r04t: 256-slot pools (build_exp/pool256.so, 4 waves per SIMD) for C4's 1/8 share at 128 / 192 / 256 pixels per
#       wave against the production 128-slot pools (128 px/wave); and C2's 1/8 share
QB="--share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2"
run() { echo "$1 $(timeout -k 10 200 env $2 python3 tools/quick_bench.py $QB | grep '^{' | tail -1)"; }
{
run main ""
run pool256_px128 "RTP_LIB_PATH=build_exp/pool256.so RTP_WAVE_PIXELS=128"
run pool256_px192 "RTP_LIB_PATH=build_exp/pool256.so RTP_WAVE_PIXELS=192"
run pool256_px256 "RTP_LIB_PATH=build_exp/pool256.so RTP_WAVE_PIXELS=256"
run main ""
} > gpurun_out/r04t_c4_s8.log 2>&1
cat gpurun_out/r04t_c4_s8.log | cut -c1-160
