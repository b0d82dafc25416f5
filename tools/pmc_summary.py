"""Summarise rocprofv3 --pmc passes for the render kernel (per launch)."""
import csv, glob, sys, collections
root = sys.argv[1]
agg = collections.defaultdict(float); launches = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "rtp_render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            launches[r["Counter_Name"]].add(r["Dispatch_Id"])
per = {k: v / max(1, len(launches[k])) for k, v in agg.items()}
for k in sorted(per): print(f"{k:28s} {per[k]:.4e}")
w = per.get("SQ_WAVES", 1)
if "SQ_INSTS_VALU" in per:
    print("VALU/wave", per["SQ_INSTS_VALU"] / w, "SALU/wave", per.get("SQ_INSTS_SALU", 0) / w)
if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per:
    print("thread-cycles per active VALU cycle", per["SQ_THREAD_CYCLES_VALU"] / per["SQ_ACTIVE_INST_VALU"])
