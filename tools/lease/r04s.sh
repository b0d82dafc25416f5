export TMPDIR=/tmp
# r04s: scheduling constants re-checked on the no-SLP build: fast-forward margin 8 / 20 (12), critical-pixel lag
#       off / 200 (100), priority balancing off; same.so = an identical rebuild (noise control); C2 and its 1/8 share
bash tools/gpu_step.sh \
 "600 r04s_ab_c2.log bash tools/ab.sh 2 main build_exp/same.so build_exp/m8.so build_exp/m20.so build_exp/crit0.so build_exp/crit200.so build_exp/prio0.so" \
 "600 r04s_ab_c2_s8.log bash tools/ab_share.sh 8 2 main build_exp/same.so build_exp/m8.so build_exp/m20.so build_exp/crit0.so build_exp/crit200.so build_exp/prio0.so"
