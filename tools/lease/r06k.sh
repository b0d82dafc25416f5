# r06k: the unchanged main.cc's -hemisphere modes (path and -direct) against the oracle;
# the port's hemisphere views with generateHemisphere's near plane (main.cc:519)
bash tools/gpu_step.sh \
 "400 r06k_main_cc_tests.log python -u -m pytest tests/test_main_unchanged.py tests/test_cpp_host.py -m gpu -v --timeout 300 --timeout-method thread"
