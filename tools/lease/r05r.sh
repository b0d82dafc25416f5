# r05r: the round's measurement set on the final C2 kernel: rocprofv3 stats of the default bench
# command, the VALU-issue counters and the HBM request-size counters of the timed instance
export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "600 r05r_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05r_prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5" \
 "400 r05r_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r05r_pv" \
 "900 r05r_pmc_bytes.log bash tools/pmc_bytes.sh gpurun_out/r05r_pb python3 tools/quick_bench.py --spp 1000 --reps 1"
python3 tools/valu_summary.py gpurun_out/r05r_pv gpurun_out/r05r_valu.json > gpurun_out/r05r_valu_summary.log 2>&1
python3 tools/bytes_summary.py gpurun_out/r05r_pb rtp_render_pool > gpurun_out/r05r_bytes_summary.log 2>&1
