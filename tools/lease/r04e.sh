export TMPDIR=/tmp
# r04e: pow5_exact (schlick) + Markstein camera divisions vs r04a: C2 at N=1 and the 1/8 share; GPU tests; stats
bash tools/gpu_step.sh \
 "400 r04e_ab_c2.log bash tools/ab.sh 2 main build_exp/r04a.so" \
 "400 r04e_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/r04a.so" \
 "900 r04e_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "300 r04e_dbg1.log python3 tools/dbg_stats.py --spp 200"
