"""Average per-launch counter values per kernel from rocprofv3
counter_collection.csv files (one directory per --pmc pass)."""
import csv
import glob
import re
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    agg = defaultdict(lambda: [0.0, set()])
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0],
                 r["Counter_Name"])
            agg[k][0] += float(r["Counter_Value"])
            agg[k][1].add(r["Dispatch_Id"])
    for (kn, cn), (v, ids) in sorted(agg.items(), key=lambda x: -x[1][0]):
        print(f"{cn:12s} {kn:40s} launches={len(ids):4d} per_launch={v / len(ids):.0f}")
