"""Per-step dynamic instruction counts of tools/lat_bench's modes from
tools/pmc_lat.sh's counter passes.  Each (mode, W) runs a 4-iteration warm
dispatch and an `iters` dispatch; the difference of their counts over
(waves x (iters - 4)) is one wave's instructions per loop step.
usage: python3 tools/lat_pmc_summary.py <outdir> <iters>"""
import collections
import csv
import glob
import json
import re
import sys

root, iters = sys.argv[1], int(sys.argv[2])
rows = collections.defaultdict(dict)  # (pass, dispatch) -> {counter: value, ...}
meta = {}
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    p = re.search(r"/p(\d+)/", f).group(1)
    for r in csv.DictReader(open(f)):
        m = re.search(r"lat_kernel<(\d+)>|lat_kernelILi(\d+)E", r["Kernel_Name"])
        if not m:
            continue
        mode = int(m.group(1) or m.group(2))
        key = (p, int(r["Dispatch_Id"]))
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[key] = (mode, int(r["Grid_Size"]))
# pair warm / timed dispatches per (pass, mode, grid) in dispatch order
groups = collections.defaultdict(list)
for key in sorted(rows):
    mode, grid = meta[key]
    groups[(key[0], mode, grid)].append(rows[key])
res = collections.defaultdict(dict)
grids = sorted({g for (_, _, g) in groups})
cus = grids[0] // 256 if grids else 1
for (p, mode, grid), ds in groups.items():
    if len(ds) < 2:
        continue
    warm, run = ds[0], ds[1]
    waves = run.get("SQ_WAVES", grid / 64)
    w = grid // 256 // cus
    for c, v in run.items():
        if c in ("SQ_WAVES", "GRBM_GUI_ACTIVE"):
            continue
        res[(mode, w)][c] = (v - warm.get(c, 0.0)) / (waves * (iters - 4))
names = {5: "ray advance (loop overhead)", 0: "closest_hit", 6: "exact scan (6 rotated-box quads)",
         7: "prefilter (12 axis quads + candidate)", 3: "shade_hit", 1: "closest_hit + shade_hit",
         2: "closest_hit, no prefilter", 4: "dependent 4-B table gather"}
cols = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD",
        "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
        "SQ_WAIT_INST_ANY"]
print("# per wave per loop step (wave-level instructions; *_CYCLES / ACTIVE / WAIT in the counters' units)")
print("mode W " + " ".join(c.replace("SQ_", "") for c in cols))
for (mode, w) in sorted(res):
    r = res[(mode, w)]
    print(f"{mode} {w} " + " ".join(f"{r.get(c, float('nan')):.1f}" for c in cols) + f"  # {names.get(mode, '')}")
json.dump({f"{m},{w}": v for (m, w), v in res.items()}, open(f"{root}/lat_pmc.json", "w"), indent=1)
