"""Summarise rocprofv3 PMC passes into profiles/<name>.json.

Usage: python tools/pmc_summary.py OUT.json FETCH_DIR WRITE_DIR
FETCH_DIR / WRITE_DIR are rocprofv3 -d directories of two separate runs with
`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (they cannot share a pass on
gfx950).  Corrections per MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            per[name].append(float(r["Counter_Value"]))
    return per


def short(name):
    """kernel name -> short label, template arguments kept"""
    import re
    m = re.search(r"(k_\w+(?:<[^>(]*>)?)\(", name)
    return m.group(1) if m else name[:60]


def main():
    out, fdir, wdir = sys.argv[1:4]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    rows = {}
    for name in set(fetch) | set(write):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        rows[short(name)] = {"dispatches": max(len(f), len(w)),
                             "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": (fb or 0) + (wb or 0)}
    fill = rows.get("k_fill<false, false>", rows.get("k_fill<false>", {}))
    res = {"note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs; FETCH x2 "
                   "(gfx950 half-count on wide streaming reads), KiB -> bytes",
           "hbm_bytes_per_launch": fill.get("hbm_bytes_per_launch"),
           "kernels": rows}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1)[:2000])


if __name__ == "__main__":
    main()
