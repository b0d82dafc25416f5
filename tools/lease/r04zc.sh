# r04zc: pixels per wave for C4's 1/8 and 1/4 shares through the tile instance (RTP_WAVE_PIXELS; default 128 at the 1/8 share)
s8="--tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2"
s4="--tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 4 --rank 0 --reps 2"
bash tools/gpu_step.sh \
 "200 r04zc_s8_def.log python3 tools/quick_bench.py $s8" \
 "200 r04zc_s8_96.log env RTP_WAVE_PIXELS=96 python3 tools/quick_bench.py $s8" \
 "200 r04zc_s8_112.log env RTP_WAVE_PIXELS=112 python3 tools/quick_bench.py $s8" \
 "200 r04zc_s8_120.log env RTP_WAVE_PIXELS=120 python3 tools/quick_bench.py $s8" \
 "200 r04zc_s4_def.log python3 tools/quick_bench.py $s4" \
 "200 r04zc_s4_96.log env RTP_WAVE_PIXELS=96 python3 tools/quick_bench.py $s4" \
 "200 r04zc_s4_112.log env RTP_WAVE_PIXELS=112 python3 tools/quick_bench.py $s4" \
 "200 r04zc_s4_128.log env RTP_WAVE_PIXELS=128 python3 tools/quick_bench.py $s4"
