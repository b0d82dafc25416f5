"""Per-launch VALU-issue summary of the render kernel from a tools/pmc_valu.sh
run (rocprofv3 csv): writes the JSON bench.py reads as `roofline_valu`.

Capacity: each of the 1024 SIMDs (256 CUs x 4) issues one wave64 VALU
instruction per 2 cycles (MI355X_MICROARCH.md, per-instruction constants:
v_fma_f32 wave64 2 cyc on SIMD-32; one wave alone 4); the cycles are the
chip's own under load, GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs), so
clock give-back under load is not counted as idle issue.

    python tools/valu_summary.py <pmc_dir> <out.json>
"""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rtp_render_pool" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
per = {}
for k, rows in agg.items():
    by = collections.defaultdict(float)
    for d, v in rows:
        by[d] += v
    per[k] = sum(by.values()) / len(by)
durs = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rtp_render_pool" in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
dur_ms = sum(durs) / len(durs)
cyc = per["GRBM_GUI_ACTIVE"] / 8
res = {
    "nx": 800, "ny": 800, "spp": 1000, "depth": 50,
    "simds": 1024, "cycles_per_wave64_valu": 2,
    "valu_insts_per_launch": per["SQ_INSTS_VALU"],
    "lanes_per_instr": per["SQ_THREAD_CYCLES_VALU"] / per["SQ_INSTS_VALU"],
    "gpu_cycles_per_launch": cyc, "kernel_ms_pmc": dur_ms, "clock_ghz": cyc / (dur_ms * 1e-3) / 1e9,
    "waves_per_launch": per.get("SQ_WAVES"),
    "frac_pmc": per["SQ_INSTS_VALU"] / (1024 * cyc / 2),
    "source": f"rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES GRBM_GUI_ACTIVE ({root})",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
