export TMPDIR=/tmp
# r04f (fresh container): HEAD (pow5_exact schlick + Markstein camera) on hardware: GPU tests, smoke,
#       A/B vs r04a at N=1 and the 1/8 share, default bench line
bash tools/gpu_step.sh \
 "900 r04f_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r04f_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 r04f_ab_c2.log bash tools/ab.sh 2 main build_exp/r04a.so" \
 "400 r04f_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/r04a.so" \
 "400 r04f_bench.log python3 -u bench.py"
