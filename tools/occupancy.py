"""Resident waves the pool kernel plans for a pixel count (device occupancy query)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (one HIP runtime)
from raytracingtherestofyourlife_amd import _lib

L = _lib.load()
L.rtp_plan_history_lanes.restype = ctypes.c_int64
L.rtp_plan_history_lanes.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int)]
for npix in [int(a) for a in sys.argv[1:]] or [640000]:
    for bvh in (0, 1):
        v, w = ctypes.c_int(), ctypes.c_int()
        lanes = L.rtp_plan_history_lanes(npix, 1000, bvh, ctypes.byref(v), ctypes.byref(w))
        print(f"npix {npix} bvh {bvh}: waves {w.value}, history lanes {lanes}")
