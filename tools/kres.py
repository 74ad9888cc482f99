"""Kernel resources (VGPRs, SGPRs, spills, scratch, LDS) of one HIP source's
gfx950 code object.  python tools/kres.py lime_amd/csrc/sort.hip [regex]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "."
out = "/tmp/kres_%s.co" % os.path.basename(src).replace(".hip", "")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                       "--cuda-device-only", "--no-gpu-bundle-output", "-Wno-pass-failed", "-c",
                       src, "-o", out])
txt = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", out], text=True)
for blk in re.split(r"\n  - (?=\.agpr_count)", txt)[1:]:
    def g(k):
        m = re.search(r"^\s+\.%s:\s+(\S+)" % k, blk, re.M)
        return m.group(1) if m else "?"
    name = g("name")
    if not re.search(filt, name):
        continue
    print("%-80s vgpr=%4s agpr=%3s sgpr=%3s vspill=%s sspill=%s scratch=%s lds=%s" % (
        name[:80], g("vgpr_count"), g("agpr_count"), g("sgpr_count"), g("vgpr_spill_count"),
        g("sgpr_spill_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size")))
