"""bench.py -- BASELINE.json's metric on its N=1 configuration (C2).

One step = the whole operator pipeline over one batch of synthetic input
already resident in HBM (unsorted, as loaded):
  device radix sort of A and B  ->  intersect count pass  ->  fill of every
  qualifying pair (16-B records, chunked through a reusable output buffer)
  ->  merge(A), merge(B)  (runs + run id of every row).
C2 = 2 x 1e8 intervals, uniform starts over hg38 primary, lengths U[50,5000]
(~1.63e10 pairs per step).  value = intervals processed per second by the
whole job (sum over ranks).

Multi-GPU (torchrun, one rank per GPU): every rank owns one coordinate shard
-- its own copy of the hg38 space with its own seeds -- and runs the same
per-GPU workload (weak scaling); shards are independent, so the data path has
no collective; a barrier brackets the timed region and the time is the max
over ranks.

Also reported: roofline of the dominant kernel (k_fill, HBM-bound) from HIP
events on the launch stream, and a CPU baseline (the oracle's restatement of
lime's sweep-line, 1 thread) on a bounded sample, rank 0 / N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rows", type=int, default=100_000_000, help="rows per set (C2: 1e8)")
    p.add_argument("--chunk", type=int, default=1 << 31, help="pairs per output chunk")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--cpu-scale", type=int, default=100,
                   help="CPU sample: C2 density on hg38/scale with n/scale rows")
    return p.parse_args()


def cpu_baseline(scale, n_full, reps=9):
    """lime's per-partition algorithms restated in C (oracle/lime_oracle.c),
    single thread, on the C2 distribution over hg38/scale with n/scale rows
    per set (same depth, so the same pairs per row); ~1 s per repetition, 9
    repetitions (~10 s of CPU work), median.  Returns intervals/s."""
    import ctypes as C

    import numpy as np

    from lime_amd import synth
    from oracle import oracle
    lens = np.array(list(synth.HG38.values())) // scale
    n = n_full // scale
    A = synth.uniform(lens, n, 0xA, 50, 5000)
    B = synth.uniform(lens, n, 0xB, 50, 5000)
    L = oracle.lib()
    P = C.POINTER
    args = []
    for X in (A, B):
        c = np.ascontiguousarray(X[0], np.int32)
        s = np.ascontiguousarray(X[1], np.int64)
        e = np.ascontiguousarray(X[2], np.int64)
        args.append((c, s, e))
    (ac, as_, ae), (bc, bs, be) = args

    def ptr(a, t):
        return a.ctypes.data_as(P(t))
    base = [n, ptr(ac, C.c_int32), ptr(as_, C.c_int64), ptr(ae, C.c_int64), None, n,
            ptr(bc, C.c_int32), ptr(bs, C.c_int64), ptr(be, C.c_int64), None, 0]
    k = L.lo_intersect(*base, 0, None, None, None, None, None)
    outs = [np.empty(k, np.int32)] + [np.empty(k, np.int64) for _ in range(4)]
    optr = [ptr(outs[0], C.c_int32)] + [ptr(o, C.c_int64) for o in outs[1:]]
    rid = np.empty(n, np.int64)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        L.lo_intersect(*base, k, *optr)
        for (c, s, e) in args:
            L.lo_merge(n, ptr(c, C.c_int32), ptr(s, C.c_int64), ptr(e, C.c_int64), None, 0,
                       None, None, None, None, ptr(rid, C.c_int64))
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    thr = cpu_baseline_threaded(L, ac, as_, ae, bc, bs, be, reps)
    return {"value": thr["value"], "unit": "intervals/s", "cores": thr["cores"], "kind": "port",
            "single_thread_value": 2 * n / t,
            "sample": f"C2 density on hg38/{scale}: 2 x {n} rows, {k} pairs, intersect + "
                      f"merge(A) + merge(B), median of {reps}; lime sweep-line restated in C "
                      f"(oracle/lime_oracle.c), {thr['cores']} threads sharded by contig "
                      f"(the Spark task per partition; largest shard {thr['max_share']:.1%} of "
                      "the rows), single_thread_value = the same on 1 thread; every call sorts "
                      "its input (qsort) inside the timed region, as the device pipeline does"}


def cpu_baseline_threaded(L, ac, as_, ae, bc, bs, be, reps):
    """The same pipeline as cpu_baseline on T host threads, sharded by contig
    (each thread owns whole contigs, rows balanced greedily), the way Spark
    runs one task per range partition (CPU baseline (2)).
    ctypes drops the GIL around each C call, so the shards run in parallel.
    T = OMP_NUM_THREADS (16 on the GPU box), at most os.cpu_count()."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    T = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 16))
    contigs = np.union1d(np.unique(ac), np.unique(bc))
    rows = {int(c): int((ac == c).sum() + (bc == c).sum()) for c in contigs}
    bins = [[] for _ in range(T)]
    load = [0] * T
    for c in sorted(rows, key=rows.get, reverse=True):
        i = load.index(min(load))
        bins[i].append(c)
        load[i] += rows[c]
    P = C.POINTER

    def ptr(a, t):
        return a.ctypes.data_as(P(t))
    shards = []
    for b in bins:
        if not b:
            continue
        ma, mb = np.isin(ac, b), np.isin(bc, b)
        A = [np.ascontiguousarray(x[ma]) for x in (ac, as_, ae)]
        B = [np.ascontiguousarray(x[mb]) for x in (bc, bs, be)]
        na, nb = len(A[0]), len(B[0])
        base = [na, ptr(A[0], C.c_int32), ptr(A[1], C.c_int64), ptr(A[2], C.c_int64), None,
                nb, ptr(B[0], C.c_int32), ptr(B[1], C.c_int64), ptr(B[2], C.c_int64), None, 0]
        k = L.lo_intersect(*base, 0, None, None, None, None, None)
        outs = [np.empty(k, np.int32)] + [np.empty(k, np.int64) for _ in range(4)]
        optr = [ptr(outs[0], C.c_int32)] + [ptr(o, C.c_int64) for o in outs[1:]]
        rid = np.empty(max(na, nb), np.int64)
        shards.append((base, k, optr, outs, A, B, rid))

    def run(sh):
        base, k, optr, _, A, B, rid = sh
        L.lo_intersect(*base, k, *optr)
        for X in (A, B):
            L.lo_merge(len(X[0]), ptr(X[0], C.c_int32), ptr(X[1], C.c_int64),
                       ptr(X[2], C.c_int64), None, 0, None, None, None, None,
                       ptr(rid, C.c_int64))
    times = []
    with ThreadPoolExecutor(len(shards)) as ex:
        for _ in range(reps):
            t0 = time.perf_counter()
            list(ex.map(run, shards))
            times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    return {"value": (len(ac) + len(bc)) / t, "cores": len(shards),
            "max_share": max(load) / max(1, sum(load))}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; --dist-backend gloo lets several ranks share one GPU
    # (rehearsal of the multi-GPU path on a 1-GPU box, boundary records on CPU)
    gpu = local % max(torch.cuda.device_count(), 1)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    comm_dev = dev
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
            comm_dev = torch.device("cpu")

    import lime_amd
    from lime_amd import synth

    ctx = lime_amd.Context(dev.index)
    # one non-default stream shared by torch and the engine: the HIP events
    # below are recorded on the stream the kernels are launched on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    space = lime_amd.Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    n = args.rows
    seed_a, seed_b = 0xA + 0x100 * rank, 0xB + 0x100 * rank

    def gen(seed):
        c = torch.empty(n, dtype=torch.int32, device=dev)
        s = torch.empty(n, dtype=torch.int32, device=dev)
        e = torch.empty(n, dtype=torch.int32, device=dev)
        ctx.synth_uniform(space, n, seed, 50, 5000, c.data_ptr(), s.data_ptr(), e.data_ptr())
        return c, s, e
    A_in, B_in = gen(seed_a), gen(seed_b)
    buf = torch.empty((args.chunk, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    fills = []  # (start event, end event, pairs) of every fill launch

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def fill_all(plan, halos=None):
        for f in range(0, plan.n, args.chunk):
            k = min(args.chunk, plan.n - f)
            e0 = ev()
            plan.fill_device(f, k, buf.data_ptr())
            fills.append((e0, ev(), k, plan.n))

    shard = None
    if world > 1:
        from lime_amd.sharded import ShardStep
        # rank r owns the r-th copy of the genome on one virtual coordinate
        # line: offset r * span; boundary exchange + merge carry over RCCL
        shard = ShardStep(ctx, space, offset=rank * space.span, comm_device=comm_dev)

    def step(phases=None):
        t = [ev()] if phases is not None else None
        A = ctx.set_from_device(space, n, *(x.data_ptr() for x in A_in))
        B = ctx.set_from_device(space, n, *(x.data_ptr() for x in B_in))
        if t is not None:
            t.append(ev())
        if shard is not None:
            out = shard.run(A, B, on_pairs=fill_all)
            for h in (out["merge_a"], out["merge_b"], A, B):
                h.close()
            if t is not None:
                t += [ev(), ev(), ev()]
                phases.append(t)
            return out["pairs"], out["runs_a"] + out["runs_b"]
        plan = ctx.intersect(A, B)
        if t is not None:
            t.append(ev())
        fill_all(plan)
        if t is not None:
            t.append(ev())
        ma, mb = ctx.merge(A), ctx.merge(B)
        if t is not None:
            t.append(ev())
            phases.append(t)
        npairs, nruns = plan.n, ma.n + mb.n
        for h in (plan, ma, mb, A, B):
            h.close()
        return npairs, nruns

    for _ in range(args.warmup):
        step()
    fills.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    phases = []
    for i in range(args.steps):
        npairs, nruns = step(phases if i == args.steps - 1 else None)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    value = world * 2 * n / (dt / args.steps)

    # roofline of the dominant kernel (fill): algorithmic bytes per launch =
    # 16 B per pair written + 20 B per owner row consumed (lo, count, start,
    # end, row), prorated to the pairs of the launch
    fill_ms = [a.elapsed_time(b) for a, b, _, _ in fills]
    fill_bytes = [16 * k + 20 * (2 * n) * k / tot for _, _, k, tot in fills]
    avg_ms = sum(fill_ms) / len(fill_ms)
    avg_b = sum(fill_bytes) / len(fill_bytes)
    achieved = avg_b / (avg_ms * 1e-3) / 1e9
    p = phases[-1]
    if world > 1:
        breakdown = {"sort_ms": p[0].elapsed_time(p[1]),
                     "merge_halo_intersect_fill_carry_ms": p[1].elapsed_time(p[2]),
                     "fill_ms": sum(fill_ms[-(-npairs // args.chunk):])}
    else:
        breakdown = {"sort_ms": p[0].elapsed_time(p[1]), "count_ms": p[1].elapsed_time(p[2]),
                     "fill_ms": p[2].elapsed_time(p[3]), "merge_ms": p[3].elapsed_time(p[4])}

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "fill_pmc.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_scale, n)

    if rank == 0:
        line = {
            "metric": "intervals/sec for pairwise intersect+merge at 1/2/4/8 GPUs; "
                      "% of HBM peak GB/s",
            "value": value, "unit": "intervals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (counter-based splitmix64, seeds 0xA/0xB per shard)",
            "config": {"workload": "C2: sort + intersect + merge(A), merge(B); 2 x 1e8 "
                                   "intervals per GPU, uniform over hg38, len U[50,5000]",
                       "rows_per_set": n, "pairs_per_step": npairs, "runs_per_step": nruns,
                       "output_chunk_pairs": args.chunk, "parallelism": f"range-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_fill<false>", "avg_launch_ms": avg_ms,
                         "alg_bytes_per_launch": avg_b, "launches": len(fills)},
            "breakdown_ms": breakdown,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
