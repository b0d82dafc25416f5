# r04w: hiding the fast-forward's jump-table gather latency.
# build_exp/ffmask.so: gathers masked into a cached 4-KB window (wrong images, timing only: the bound);
# build_exp/pipe.so: pipelined batches (RTP_PIPE_FF=1), bit-exact (digests against main)
bash tools/gpu_step.sh \
 "200 r04w_digest_main.log python3 tools/lib_digest.py --spp 64" \
 "200 r04w_digest_pipe.log env RTP_LIB_PATH=build_exp/pipe.so python3 tools/lib_digest.py --spp 64" \
 "200 r04w_digest_main_s.log python3 tools/lib_digest.py --nx 1920 --ny 1080 --spp 256 --begin 0 --count 259200" \
 "200 r04w_digest_pipe_s.log env RTP_LIB_PATH=build_exp/pipe.so python3 tools/lib_digest.py --nx 1920 --ny 1080 --spp 256 --begin 0 --count 259200" \
 "400 r04w_ab_c4s8.log env QB_ARGS='--share --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0' bash tools/ab.sh 2 main build_exp/ffmask.so build_exp/pipe.so" \
 "400 r04w_ab_c2.log bash tools/ab.sh 2 main build_exp/ffmask.so build_exp/pipe.so" \
 "400 r04w_ab_c2s8.log env QB_ARGS='--share --nx 800 --ny 800 --spp 1000 --depth 50 --world 8 --rank 0' bash tools/ab.sh 2 main build_exp/ffmask.so build_exp/pipe.so"
