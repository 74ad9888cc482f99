"""HBM bytes per kernel from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate runs, MI355X_MICROARCH.md "HBM"), written as the JSON
that bench.py reads its roofline "traffic" from, with its provenance.

  python tools/pmc_json.py OUT.json FETCH_DIR WRITE_DIR --commit SHA --cmd "..."
      [--key KERNEL] [--steps N] [--exclude SUBSTR ...]

Counters: FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950
counts half the bytes of a wide coalesced streaming read).  --key names the
dominant kernel whose per-launch bytes become "hbm_bytes_per_launch";
--steps N divides the bytes of every kernel not excluded (e.g. the input
generator) by the N steps the profiled command ran, as "hbm_bytes_per_step".
"""
import argparse
import csv
import glob
import json
import re
import time
from collections import defaultdict


def load(d):
    agg = defaultdict(lambda: [0.0, set()])
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
            k = k.replace("lime::", "")
            agg[k][0] += float(r["Counter_Value"])
            agg[k][1].add(r["Dispatch_Id"])
    return agg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("fetch")
    p.add_argument("write")
    p.add_argument("--commit", required=True)
    p.add_argument("--cmd", required=True)
    p.add_argument("--key")
    p.add_argument("--steps", type=int, default=0)
    p.add_argument("--exclude", nargs="*", default=[])
    a = p.parse_args()
    fe, wr = load(a.fetch), load(a.write)
    kernels = {}
    step_bytes = 0.0
    for k in sorted(set(fe) | set(wr)):
        nd = max(len(fe[k][1]) if k in fe else 0, len(wr[k][1]) if k in wr else 0)
        f = 2 * 1024 * fe[k][0] if k in fe else 0.0
        w = 1024 * wr[k][0] if k in wr else 0.0
        kernels[k] = {"dispatches": nd, "fetch_bytes_per_launch": f / nd,
                      "write_bytes_per_launch": w / nd, "hbm_bytes_per_launch": (f + w) / nd,
                      "hbm_bytes_total": f + w}
        if not any(x in k for x in a.exclude):
            step_bytes += f + w
    out = {"note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate runs; FETCH x2 "
                   "(gfx950 counts half of a wide streaming read), KiB -> bytes",
           "provenance": {"commit": a.commit, "command": a.cmd,
                          "generated": time.strftime("%Y-%m-%d %H:%M:%S"),
                          "fetch_dir": a.fetch, "write_dir": a.write},
           "kernels": kernels}
    if a.key:
        hit = [k for k in kernels if k == a.key] or [k for k in kernels if a.key in k]
        if not hit:
            raise SystemExit(f"kernel {a.key!r} not in the profile: {sorted(kernels)}")
        out["key_kernel"] = hit[0]
        out["hbm_bytes_per_launch"] = kernels[hit[0]]["hbm_bytes_per_launch"]
    if a.steps:
        out["steps_profiled"] = a.steps
        out["excluded"] = a.exclude
        out["hbm_bytes_per_step"] = step_bytes / a.steps
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
