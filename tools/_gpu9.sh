bash tools/gpu_step.sh \
 "300 r03i_slot80.log python -u tools/slot_plan.py --pixels-per-wave 80" \
 "300 r03i_slot125.log python -u tools/slot_plan.py --pixels-per-wave 125" \
 "300 r03i_spec_tests.log env RTP_LIB_PATH=variants/spec_ff.so python -u -m pytest tests/test_golden.py -x -q --timeout 240 --timeout-method thread -m gpu -k full_frame" \
 "600 r03i_ab1.log bash tools/ab_c2_tiles.sh 3 main variants/spec_ff.so" \
 "600 r03i_ab8.log bash tools/ab_share.sh 8 3 main variants/spec_ff.so variants/noff.so" \
 "600 r03i_ab2.log bash tools/ab_share.sh 2 2 main variants/spec_ff.so"
