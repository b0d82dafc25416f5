export TMPDIR=/tmp
# r04q: bench at N = 1 through the default contiguous launch (bench.py --n1-launch contig), its rocprof stats,
#       VALU and HBM-byte counters of that instance; the tile instance's bench line beside it
mkdir -p gpurun_out/r04q
bash tools/gpu_step.sh \
 "400 r04q_bench.log python3 -u bench.py" \
 "400 r04q_bench_tiles.log python3 -u bench.py --n1-launch tiles --cpu-budget 0 --cpu-budget-mt 0" \
 "400 r04q_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04q_prof -o bench --output-format csv -- python3 -u bench.py --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r04q_pmc_valu.log bash tools/pmc_valu.sh gpurun_out/r04q_pv" \
 "900 r04q_pmc_bytes.log bash tools/pmc_bytes.sh gpurun_out/r04q_pb python3 tools/quick_bench.py --spp 1000 --reps 1"
