# r06s: the final round-6 tree: GPU suite, smoke, bench, rocprof stats of the bench, and the
# reference's unchanged main.cc rendering C2 once (its own "Elapsed time": setup, render,
# NormalizeFunctor, save() of the P3 PNM)
export TMPDIR=/tmp
bash tools/gpu_step.sh \
 "1000 r06s_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r06s_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r06s_bench.log python3 -u bench.py --steps 20 --warmup 5" \
 "500 r06s_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r06s_prof -o r06s -- python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --cpu-budget-mt 0" \
 "300 r06s_main_cc.log bash -c 'mkdir -p /tmp/mcc && cd /tmp/mcc && $GRAFT_REPO_ROOT/examples/main_cc -x 800 -y 800 -samplecount 1000 -raydepth 50 && ls -la /tmp/mcc'"
