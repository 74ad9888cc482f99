"""Per-kernel summary (calls, avg us, total ms) of a rocprofv3 --stats run:
python tools/kstats.py DIR_OR_CSV  (the kernel_stats.csv rocprofv3 writes)."""
import csv
import glob
import os
import sys

p = sys.argv[1]
if os.path.isdir(p):
    c = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
    if not c:
        sys.exit("no kernel_stats.csv under " + p)
    p = c[0]
print(p)
print("%-74s %6s %10s %10s" % ("kernel", "calls", "avg_us", "total_ms"))
for r in csv.DictReader(open(p)):
    name = r["Name"].replace("(anonymous namespace)::", "")
    print("%-74s %6s %10.1f %10.2f" % (name[:74], r["Calls"], float(r["AverageNs"]) / 1e3,
                                        float(r["TotalDurationNs"]) / 1e6))
