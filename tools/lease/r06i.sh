# r06i: the point-field fix (89 values): every -direct test, the unchanged main.cc, smoke
bash tools/gpu_step.sh \
 "600 r06i_gputests.log python -u -m pytest tests/test_gpu_direct.py tests/test_main_unchanged.py tests/test_cpp_host.py tests/test_golden.py tests/test_direct.py -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r06i_smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'"
