bash tools/gpu_step.sh \
 "300 r03a_fullframe.log python -u -m pytest tests/test_golden.py -k c2_full -x -v --timeout 240 --timeout-method thread -m gpu" \
 "300 r03a_bench_base.log python -u bench.py --steps 10 --warmup 2" \
 "240 r03a_setup_default.log python -u tools/setup_cost.py" \
 "240 r03a_setup_notables.log env RTP_FF_TABLES=0 python -u tools/setup_cost.py" \
 "240 r03a_setup_chain.log env RTP_FF_DIRECT=0 python -u tools/setup_cost.py" \
 "240 r03a_share8.log python -u tools/quick_bench.py --tiles --spp 1000 --world 8 --rank 0 --reps 3" \
 "240 r03a_share8_notables.log env RTP_FF_TABLES=0 python -u tools/quick_bench.py --tiles --spp 1000 --world 8 --rank 0 --reps 3" \
 "240 r03a_share4.log python -u tools/quick_bench.py --tiles --spp 1000 --world 4 --rank 0 --reps 3" \
 "240 r03a_share2.log python -u tools/quick_bench.py --tiles --spp 1000 --world 2 --rank 0 --reps 3"
