# r05v: AMDGPU backend options (early if-conversion, scheduler occupancy/latency bias, relaxed occupancy, no pre-RA opts)
bash tools/gpu_step.sh \
 "1200 r05v_ab_c2.log bash tools/ab.sh 2 build_exp/lib_m_base.so build_exp/lib_f_ifcvt.so build_exp/lib_f_bias0.so build_exp/lib_f_bias100.so build_exp/lib_f_relaxocc.so build_exp/lib_f_noprera.so"
