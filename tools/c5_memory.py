"""Device memory of C5's binned AND (lime_amd.h): 8 x 1.25e8
unsorted rows (len U[10,40], seeds 0x50..0x57, as bench.py's C5) ->
lime_bitset_and_from_device.  Prints one JSON line: the rows' bytes, the
engine pool's bytes before / after building the bitset (the bins it keeps),
after painting the words, after lime_bitset_drop_bins and after destroying
it, and the device's used bytes (hipMemGetInfo) at each point.
  python tools/c5_memory.py [--rows 125000000]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=125_000_000)
    a = p.parse_args()
    import torch

    import lime_amd
    from lime_amd import synth
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = lime_amd.Context(0)
    space = lime_amd.Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    k, n = 8, a.rows
    ins = []
    for i in range(k):
        c, s, e = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3))
        ctx.synth_uniform(space, n, 0x50 + i, 10, 40, c.data_ptr(), s.data_ptr(), e.data_ptr())
        ins.append((c, s, e))
    torch.cuda.synchronize(dev)

    def used():
        free, total = torch.cuda.mem_get_info(dev)
        return total - free

    def mark(tag):
        ctx.synchronize()
        live, peak = ctx.pool_live_bytes(reset_peak=True)
        out[tag] = {"live": live, "peak": peak, "pool_held": ctx.pool_bytes(),
                    "device_used": used()}

    out = {"rows": k * n, "row_bytes": 12 * k * n}
    mark("start")
    bs = ctx.bitset_and_from_device(space, [(n, *(x.data_ptr() for x in X)) for X in ins])
    mark("binned")  # the bitset keeps every set's bins; peak = the build's
    runs = ctx.bitset_runs(0, bs)
    out["runs"] = runs.n
    mark("runs")  # peak = the extraction's, live + its result
    runs.close()
    bs.popcount()  # paints the words
    mark("painted")
    bs.drop_bins()
    mark("dropped")
    bs.close()
    mark("closed")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
