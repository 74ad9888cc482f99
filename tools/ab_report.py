"""Summarise tools/ab.sh output: per variant and run, ms/step and the
average duration of the main kernels (from the rocprofv3 db)."""
import glob
import json
import os
import sqlite3
import sys

tag = sys.argv[1]
KS = ["k_fill<", "k_count", "k_windows", "k_scatter", "k_hist", "k_prep", "k_merge_scan"]
for txt in sorted(glob.glob(f"gpurun_out/{tag}_*.txt")):
    line = [ln for ln in open(txt) if ln.startswith('{"metric"')]
    ms = json.loads(line[0])["ms_per_step"] if line else float("nan")
    dbs = glob.glob(txt[:-4] + "/**/*.db", recursive=True)
    row = {}
    if dbs:
        c = sqlite3.connect(dbs[0])
        for name, avg in c.execute("select name, avg(end-start)/1e6 from kernels group by name"):
            for k in KS:
                if k in name:
                    row[k] = row.get(k, 0) + avg
    print("%-40s %7.2f  " % (os.path.basename(txt), ms) +
          "  ".join("%s=%.3f" % (k.split("<")[0], row[k]) for k in KS if k in row))
