# r05p: instruction-cache counters, HEAD vs the vertical-face prefilter build
bash tools/gpu_step.sh "600 r05p_icache.log bash tools/pmc_icache.sh gpurun_out/r05p_ic build_exp/lib_head.so main"
for d in gpurun_out/r05p_ic/*/; do echo "== $d"; find $d -name "*counter_collection.csv" -exec python3 -c "
import csv,sys,collections
agg=collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'rtp_render_pool' in r['Kernel_Name']: agg[r['Counter_Name']]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print(k, '%.4e'%v)
" {} \; ; done > gpurun_out/r05p_icache_summary.txt 2>&1
