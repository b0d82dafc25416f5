bash tools/gpu_step.sh \
 "900 r03m_ab1.log bash tools/ab_c2_tiles.sh 3 main variants/lrtf.so variants/lrtf800.so" \
 "300 r03m_chain1_lrtf.log env RTP_LIB_PATH=variants/lrtf.so python -u tools/chain_floor.py" \
 "600 r03m_ab2.log env RTP_WAVE_PIXELS=96 bash tools/ab_share.sh 2 2 main variants/lrtf.so variants/lrtf800.so" \
 "600 r03m_ab4.log env RTP_WAVE_PIXELS=96 bash tools/ab_share.sh 4 2 main variants/lrtf.so variants/lrtf800.so" \
 "300 r03m_parity.log env RTP_LIB_PATH=variants/lrtf.so python -u -m pytest tests/test_golden.py -x -q --timeout 240 --timeout-method thread -m gpu -k full_frame"
