"""Step-by-step probe of bench.py's sharded C2 step at one rank over RCCL:
each stage synchronised and timed, one line printed per stage (a hang names
its stage), the routed sets' statistics compared with the unsharded build.
  python tools/shard_diag.py [rows] [--gloo]"""
import os
import socket
import sys
import time


def main():
    rows = int(next((a for a in sys.argv[1:] if a.isdigit()), "100000000"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1]))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()

    def say(msg):
        torch.cuda.synchronize(dev)
        print(f"[{time.time() - t0:7.2f}s] {msg}", flush=True)
    gloo = "--gloo" in sys.argv
    if gloo:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=dev)
    say(f"init ({'gloo' if gloo else 'nccl'}), rows {rows}")
    import lime_amd
    from lime_amd import synth
    from lime_amd.sharded import ShardStep
    ctx = lime_amd.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    space = lime_amd.Space(list(synth.HG38.keys()), list(synth.HG38.values()))

    def gen(seed):
        c, s, e = (torch.empty(rows, dtype=torch.int32, device=dev) for _ in range(3))
        ctx.synth_uniform_rows(space, 0, rows, seed, 50, 5000, c.data_ptr(), s.data_ptr(),
                               e.data_ptr())
        return c, s, e
    A_in, B_in = gen(0xA), gen(0xB)
    say("inputs")
    shard = ShardStep(ctx, space, comm_device=torch.device("cpu") if gloo else None,
                      shared_stream=True)
    shard.plan_splits([(rows, A_in[0].data_ptr(), A_in[1].data_ptr()),
                       (rows, B_in[0].data_ptr(), B_in[1].data_ptr())])
    say(f"splits {shard.splits}")
    ref = ctx.set_from_device(space, rows, *(x.data_ptr() for x in A_in))
    say(f"unsharded A: n {ref.n} stats {ref.stats()}")
    ref.close()
    # the route's three stages, each checked (at one rank the exchange is the
    # identity: recv must equal the send buffer)
    from lime_amd import dist as ld
    buf = torch.empty((rows, 3), dtype=torch.int32, device=dev)
    counts = ctx.route_rows_interleaved(space, rows, *(x.data_ptr() for x in A_in),
                                        shard.splits, 3, buf.data_ptr(), clip=False, cap=rows)
    w = (buf[:, 1] - buf[:, 0]).to(torch.int64)
    say(f"route: counts {counts} widths [{int(w.min())}, {int(w.max())}] "
        f"rows ok {bool((buf[:, 2] == torch.arange(rows, device=dev, dtype=torch.int32)).all())}")
    recv, rc = ld.exchange_rows(buf, counts, None, torch.device("cpu") if gloo else None)
    say(f"exchange: {tuple(recv.shape)} equal {bool(torch.equal(recv, buf))}")
    if not torch.equal(recv, buf):
        bad = (recv != buf).any(dim=1).nonzero().flatten()
        say(f"  {bad.numel()} rows differ, first {bad[:4].tolist()} last {bad[-4:].tolist()}")
    cols = [torch.empty(rows, dtype=torch.int32, device=dev) for _ in range(3)]
    ctx.deinterleave(rows, 3, recv.data_ptr(), *(c.data_ptr() for c in cols))
    say(f"deinterleave: equal {[bool(torch.equal(cols[j], recv[:, j])) for j in range(3)]}")
    del buf, recv, cols, w
    for it in range(2):
        A = shard.load(rows, *(x.data_ptr() for x in A_in))
        say(f"[{it}] load A: n {A.n} stats {A.stats()}")
        B = shard.load(rows, *(x.data_ptr() for x in B_in))
        say(f"[{it}] load B: n {B.n} stats {B.stats()}")
        ma, mb = ctx.merge(A), ctx.merge(B)
        say(f"[{it}] merges: {ma.n} {mb.n}")
        plan = ctx.intersect(A, B, 0, a_owned=A.n, b_owned=B.n)
        say(f"[{it}] intersect (owned): {plan.n} pairs")
        plan.close()
        plan = ctx.intersect(A, B)
        say(f"[{it}] intersect: {plan.n} pairs")
        plan.close()
        out = shard.run(A, B)
        say(f"[{it}] run: pairs {out['pairs']} runs {out['runs_a']} {out['runs_b']}")
        for h in (out["merge_a"], out["merge_b"], ma, mb, A, B):
            h.close()
    dist.destroy_process_group()
    say("done")


if __name__ == "__main__":
    main()
