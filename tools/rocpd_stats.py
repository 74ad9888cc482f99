"""Per-kernel stats (calls, total / average ns) from a rocprofv3 rocpd .db,
in the shape of rocprofv3's kernel_stats.csv (for boxes whose rocprofv3
writes only the database)."""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows = db.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                  f"group by {name} order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage"')
for n, c, t, a in rows:
    short = re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0]
    print(f'"{short}",{c},{t},{a:.1f},{100 * t / tot:.2f}')
