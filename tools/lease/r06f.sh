set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 tools/ab.sh 3 main build_exp/lib_base.so > gpurun_out/r06f_ab_c2.txt 2>&1
