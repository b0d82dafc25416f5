# r04v: two paths per lane. lat_bench modes 11-13 against 0/1; the pair kernel's
# parity tests; C4 shares (rank 0 of 8 and of 4) with RTP_PAIR=0/1
bash tools/gpu_step.sh \
 "300 r04v_lat.log tools/lat_bench 2000 13 0 11 1 12" \
 "300 r04v_pair_tests.log python -u -m pytest tests/test_gpu_pair.py -x -v --timeout 120 --timeout-method thread" \
 "300 r04v_s8_pair0.log env RTP_PAIR=0 python3 tools/quick_bench.py --share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04v_s8_pair1.log env RTP_PAIR=1 python3 tools/quick_bench.py --share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 2" \
 "300 r04v_s4_pair1.log env RTP_PAIR=1 python3 tools/quick_bench.py --share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 4 --rank 0 --reps 2" \
 "300 r04v_s4_pair0.log env RTP_PAIR=0 python3 tools/quick_bench.py --share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 4 --rank 0 --reps 2"
