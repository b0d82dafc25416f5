"""Per-dispatch request-size counters from tools/pmc_bytes.sh, and the bytes they imply."""
import collections
import csv
import glob
import sys

root, pattern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
per = collections.defaultdict(lambda: collections.defaultdict(float))
count = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        if pattern not in name:
            continue
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        count[name][r["Counter_Name"]].add(r["Dispatch_Id"])
for name, cs in per.items():
    c = {k: v / max(1, len(count[name][k])) for k, v in cs.items()}  # per launch
    rd = 32 * c.get("TCC_EA0_RDREQ_32B", 0) + 64 * c.get("TCC_EA0_RDREQ_64B", 0) + 128 * c.get("TCC_EA0_RDREQ_128B", 0)
    print(name)
    for k in sorted(c):
        print(f"  {k:24s} {c[k]:.4e}")
    print(f"  read bytes by request size  {rd:.4e}")
    print(f"  FETCH_SIZE bytes            {1024 * c.get('FETCH_SIZE', 0):.4e}")
    print(f"  WRITE_SIZE bytes            {1024 * c.get('WRITE_SIZE', 0):.4e}")
