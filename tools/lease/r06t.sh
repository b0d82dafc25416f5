# r06t: the overlapped tree reduce's device path (communication stream, events) with ranks as
# objects in one process and an in-process hub for the transfers
bash tools/gpu_step.sh \
 "300 r06t_tree_device.log python -u -m pytest tests/test_gpu_tree_reduce.py -m gpu -v --timeout 200 --timeout-method thread"
