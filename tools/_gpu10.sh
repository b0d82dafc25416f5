export TMPDIR=/tmp
timeout -k 10 120 python3 tools/scene_cost.py > gpurun_out/r03j_scene_cost.log 2>&1 || true
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/r03j_list_avail.log 2>&1 || true
QB_ARGS="--tiles --spp 1000 --world 8 --rank 0 --ff-tables auto" timeout -k 10 900 bash tools/ab_env.sh 2 "RTP_FF_AUTO_SAMPLES=1" "RTP_FF_AUTO_SAMPLES=1,1000000000000000" "RTP_FF_AUTO_SAMPLES=1000000000000000" > gpurun_out/r03j_ffpol8.log 2>&1 &&
QB_ARGS="--tiles --spp 1000 --world 2 --rank 0 --ff-tables auto" timeout -k 10 900 bash tools/ab_env.sh 1 "RTP_FF_AUTO_SAMPLES=1" "RTP_FF_AUTO_SAMPLES=1,1000000000000000" "RTP_FF_AUTO_SAMPLES=1000000000000000" > gpurun_out/r03j_ffpol2.log 2>&1
