"""Per-kernel summary (calls, avg ms, total ms) of a rocprofv3 results db."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = ("select name, count(*), avg(end-start)/1e6, sum(end-start)/1e6 from kernels "
     "group by name order by sum(end-start) desc")
print("%-70s %6s %10s %10s" % ("kernel", "calls", "avg_ms", "total_ms"))
for r in c.execute(q):
    print("%-70s %6d %10.4f %10.2f" % (r[0][:70], r[1], r[2], r[3]))
