# r04zf: rocprofv3 kernel statistics of bench.py's N > 1 render on one GPU: rank 0 of 8's C4 share through the tile instance
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
bash tools/gpu_step.sh \
 "400 r04zf_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04zf_prof -o share --output-format csv -- python3 tools/quick_bench.py --tiles --nx 1920 --ny 1080 --spp 4096 --depth 50 --world 8 --rank 0 --reps 3"
