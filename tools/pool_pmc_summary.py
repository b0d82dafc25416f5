"""Per-launch SQ counters of the render kernel (tools/pmc_pool.sh) and the
same per live bounce (lane-level: quick_bench's live-bounce count; the tile
instances carry no live counters, so their L comes from the contiguous
launches' fixture values below) and per sample.
usage: python3 tools/pool_pmc_summary.py <outdir> <workload>..."""
import csv
import glob
import json
import sys

root = sys.argv[1]
# samples per launch, mean live bounces per sample (C2 L from the full-frame fixture; C4 / C5 from r04u/r05a)
W = {"c2": (640000 * 1000, 3.706576), "c2s8": (80128 * 1000, 3.706576), "c4s8": (259200 * 4096, 3.7045),
     "c5s8": (8294400 * 2048, 3.7065)}
out = {}
for wl in sys.argv[2:]:
    tot = {}
    for f in sorted(glob.glob(f"{root}/{wl}/p*/**/*counter_collection.csv", recursive=True)):
        per = {}
        for r in csv.DictReader(open(f)):
            if "rtp_render_pool" not in r["Kernel_Name"]:
                continue
            per.setdefault(r["Dispatch_Id"], {})
            c = r["Counter_Name"]
            per[r["Dispatch_Id"]][c] = per[r["Dispatch_Id"]].get(c, 0.0) + float(r["Counter_Value"])
        if per:
            last = per[sorted(per, key=int)[-1]]  # the timed render (quick_bench --reps 1: the only one)
            tot.update(last)
    smp, L = W[wl]
    bounces = smp * L
    row = {k: v for k, v in tot.items()}
    row["per_live_bounce"] = {k: v / bounces * 64 for k, v in tot.items() if k.startswith("SQ_INSTS")}
    out[wl] = row
    print(f"== {wl}: {smp:.3e} samples, {bounces:.3e} live bounces")
    for k in sorted(tot):
        extra = f"   x64/bounce {tot[k] / bounces * 64:8.1f}" if k.startswith("SQ_INSTS") else ""
        print(f"  {k:24s} {tot[k]:.4e}{extra}")
json.dump(out, open(f"{root}/pool_pmc.json", "w"), indent=1)
