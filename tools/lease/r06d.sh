set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_prefilter.py tests/test_golden.py -k "prefilter or box or c2_full or hip_reproduces" > gpurun_out/r06d_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r06d_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 tools/ab.sh 3 main build_exp/lib_base.so > gpurun_out/r06d_ab_c2.txt 2>&1
