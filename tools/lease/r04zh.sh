# r04zh: where C3's time goes: the stats build's per-region cycles on C3's scene (800x800 x 8 spp: no stealing) and C2 for comparison
bash tools/gpu_step.sh \
 "300 r04zh_c3_stats.log env RTP_DEBUG_STATS=1 python3 tools/dbg_stats.py --variant 3 --n 800 --spp 8" \
 "300 r04zh_c2_stats.log env RTP_DEBUG_STATS=1 python3 tools/dbg_stats.py --variant 0 --n 800 --spp 50"
