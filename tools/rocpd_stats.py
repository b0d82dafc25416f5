"""Kernel statistics (calls, total / average / min / max duration) from a
rocprofv3 run's rocpd database (<dir>/*_results.db), as the CSV the
--stats option writes for csv output.  usage: tools/rocpd_stats.py <db> <out.csv>"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = list(c.execute("""select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start),
                                min(d.end - d.start), max(d.end - d.start)
                         from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                         group by s.kernel_name order by 3 desc"""))
total = sum(r[2] for r in rows)
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 3), mn, mx])
print(open(out).read())
