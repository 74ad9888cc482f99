"""fill_exp.py -- timing experiments on the C2 fill kernel (not part of the
product): fill launches of one 2^31-record chunk vs the checksum-only mode
of the same kernel (no stores), to split the fill's time into its store
stream and its staging / LDS work.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lime_amd  # noqa: E402
from lime_amd import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = lime_amd.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    space = lime_amd.Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    n = int(os.environ.get("ROWS", "100000000"))

    def gen(seed):
        c, s, e = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3))
        ctx.synth_uniform(space, n, seed, 50, 5000, c.data_ptr(), s.data_ptr(), e.data_ptr())
        return ctx.set_from_device(space, n, c.data_ptr(), s.data_ptr(), e.data_ptr())
    A, B = gen(0xA), gen(0xB)
    plan = ctx.intersect(A, B)
    chunk = 1 << 31
    buf = torch.empty((chunk, 4), dtype=torch.int32, device=dev)

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e
    out = {"pairs": plan.n}
    ts = []
    for r in range(5):
        f = (r * chunk) % (plan.n - chunk)
        a = ev()
        plan.fill_device(f, chunk, buf.data_ptr())
        b = ev()
        ts.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts[1:])
    out["fill_chunk_ms"] = ms[len(ms) // 2]
    out["fill_GBps"] = chunk * 16 / (out["fill_chunk_ms"] * 1e-3) / 1e9
    ts = []
    for r in range(3):
        a = ev()
        plan.checksum()
        b = ev()
        ts.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts[1:])
    out["checksum_all_ms"] = ms[0]
    out["checksum_per_chunk_ms"] = ms[0] * chunk / plan.n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
