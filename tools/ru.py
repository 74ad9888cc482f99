"""Per-kernel VGPRs / spills / LDS / occupancy from hipcc's
-Rpass-analysis=kernel-resource-usage remarks:
  hipcc ... -Rpass-analysis=kernel-resource-usage -c x.hip 2>&1 | python tools/ru.py [regex]"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
rows, cur = [], None
for ln in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|"
                  r"Occupancy \[waves/SIMD\]): (\S+)", ln)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
except OSError:
    dem = names
for r, d in zip(rows, dem):
    d = d.replace("lime::(anonymous namespace)::", "")
    if pat and not pat.search(d):
        continue
    print("%-70s vgpr %4s spill %3s lds %6s occ %s" % (d[:70], r.get("VGPRs"), r.get("VGPRs Spill"),
                                                      r.get("LDS Size"), r.get("Occupancy")))
