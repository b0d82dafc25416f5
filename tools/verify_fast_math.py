"""Exhaustive device checks of fast reciprocal / sqrt sequences."""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import raytracingtherestofyourlife_amd as rtp
dev = rtp.Device(0)
res = {}
ranges = {"pos [2^-40, 2^40]": (2.0**-40, 2.0**40), "neg [-2^40, -2^-40]": (-2.0**-40, -2.0**40),
          "pos normals [2^-126, 2^127]": (2.0**-126, 2.0**127), "neg normals": (-2.0**-126, -2.0**127)}
for kind in range(5):
    for name, (lo, hi) in ranges.items():
        if kind >= 2 and lo < 0: continue
        t = time.time()
        bad, first = dev.verify_fast_math(kind, lo, hi)
        res[f"kind{kind} {name}"] = dict(mismatches=bad, first_bad=hex(first), first_val=float(np.uint32(first).view(np.float32)), s=round(time.time()-t, 2))
        print(f"kind{kind} {name}: {bad} mismatches, first {hex(first)}", flush=True)
json.dump(res, open("gpurun_out/fast_math.json", "w"), indent=1)
