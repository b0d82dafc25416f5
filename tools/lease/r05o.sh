# r05o: candidate / fall-back rates of the vertical-face prefilter per ray population
bash tools/gpu_step.sh \
 "300 r05o_rate_vert.log python3 tools/prefilter_rate.py" \
 "300 r05o_rate_novert.log env RTP_PREFILTER_VERT=0 python3 tools/prefilter_rate.py"
