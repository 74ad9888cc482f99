"""bench.py -- BASELINE.json's metric on its configurations.

--workload c2 (default; the headline metric "intervals/sec for pairwise
intersect+merge"): one step = the whole operator pipeline over one batch of
synthetic input already resident in HBM (unsorted, as loaded):
  N = 1:  device radix sort of A and B -> intersect count pass -> fill of
          every qualifying pair (16-B records, chunked through a reusable
          output buffer) -> merge(A), merge(B) (runs + run id of every row).
  N > 1:  ONE C2 input (the same 2 x 1e8 rows) range-sharded over the N
          ranks (strong scaling): every rank starts from its 1/N slice of the
          unsorted rows; route to owner shards (device counting scatter +
          all_to_all over RCCL) -> sort -> local merges -> device halo
          exchange -> owned intersect count + fill -> merge carry
          (lime_amd.sharded.ShardStep).
C2 = 2 x 1e8 intervals, uniform starts over hg38 primary, lengths U[50,5000]
(~1.63e10 pairs per step).

--workload c5: BASELINE C5, the 8-way intersection of 8 x 1.25e8 rows (len
U[10,40], seeds 0x50..0x57) over hg38: every rank holds its 1/N slice of every
set; rows routed to the shard(s) they overlap, clipped (exact for per-base
algebra), bit-per-base sets painted per shard window, AND-ed, runs extracted,
boundary carry (lime_amd.sharded.ShardedAnd; no collective at N = 1).

value = intervals processed per second by the whole job; the time is the
max over ranks of the timed region, bracketed by barriers.

Also reported: the roofline of the dominant kernel (c2: k_fill, HBM-bound,
HIP events on the launch stream; c5: the whole step against its
algorithmic bytes 12 B per row + 8 bitsets of G/8) and a CPU baseline (the
oracle's restatement of lime's algorithm on a bounded sample), rank 0 /
N = 1 only.
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
    p.add_argument("--workload", default="c2", choices=["c2", "c5", "c3", "sub"],
                   help="c2: intersect + merge (the metric); c5: 8-way AND; c3: merge side "
                        "(sort + merge + carry + run ids + complement) of C3's pile-ups; sub: "
                        "subtract (lime mode) of the 1B-interval sets (2 x 5e8, len U[10,40])")
    p.add_argument("--no-ops", action="store_true",
                   help="c2: skip the short c3 / sub lines reported under 'operators'")
    p.add_argument("--ops-steps", type=int, default=3)
    p.add_argument("--rows", type=int, default=None,
                   help="rows per set (C2: 1e8; C5: 1.25e8, 8 sets)")
    p.add_argument("--chunk", type=int, default=1 << 31, help="pairs per output chunk")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--cpu-scale", type=int, default=100,
                   help="CPU sample: C2 density on hg38/scale with n/scale rows")
    p.add_argument("--sharded", action="store_true",
                   help="c2 at N = 1 through the sharded step (a one-rank process group): "
                        "the route / exchange / carry overheads the N > 1 runs pay, measured "
                        "on one GPU (a diagnostic, not the metric's N = 1 line)")
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


def c5_cpu_baseline(scale, per_full, k=8, reps=3):
    """lime's fold of intersect over merged operands
    restated in C (oracle/lime_oracle.c, contig-sharded threads), on C5's
    density over hg38/scale with per/scale rows per set; sort included."""
    import numpy as np

    from lime_amd import synth
    from oracle import oracle
    lens = np.array(list(synth.HG38.values())) // scale
    n = per_full // scale
    sets = [synth.uniform(lens, n, 0x50 + i, 10, 40) for i in range(k)]
    nc = len(lens)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        merged = [oracle.merge_mt(nc, X) for X in sets]
        cur = merged[0]
        for m in merged[1:]:
            ix = oracle.intersect_mt(nc, (cur["contig"], cur["start"], cur["end"]),
                                     (m["contig"], m["start"], m["end"]), records=True)
            cur = {q: ix[q] for q in ("contig", "start", "end")}
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    thr = oracle.threads()
    return {"value": k * n / t, "unit": "intervals/s", "cores": thr, "kind": "port",
            "sample": f"C5 density on hg38/{scale}: {k} x {n} rows, merge of every set then "
                      f"the fold of intersect over the merged operands (Appendix A.4), median "
                      f"of {reps}; restated in C (oracle/lime_oracle.c), {thr} threads sharded "
                      "by contig; every merge sorts its input inside the timed region"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, script=None, argv=None):
    """`bench.py --gpus N` without a launcher: start N fresh child processes
    of this script, one rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, rendezvous on 127.0.0.1), before this process has touched
    the GPU (torch is not even imported here).  Rank 0's stdout is relayed
    line by line; its JSON line must report n_gpus == N.  If any child fails,
    the others are terminated and its exit status is returned."""
    import subprocess
    import threading
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)]
                                      + list(sys.argv[1:] if argv is None else argv),
                                      env=env, stdout=subprocess.PIPE if r == 0 else None,
                                      text=True))
    lines = []

    def stop_children(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        sys.exit(128 + signum)
    import signal
    signal.signal(signal.SIGTERM, stop_children)
    signal.signal(signal.SIGINT, stop_children)

    def relay():
        for ln in procs[0].stdout:
            lines.append(ln)
            sys.stdout.write(ln)
            sys.stdout.flush()
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    if rc:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"bench.py: a rank exited with status {rc}; the others were stopped",
              file=sys.stderr)
        return rc if rc > 0 else 1
    th.join(timeout=30)
    rec = None
    for ln in lines:
        try:
            rec = json.loads(ln)
        except ValueError:
            continue
    if rec is None or rec.get("n_gpus") != n:
        print(f"bench.py: rank 0 did not report n_gpus == {n}", file=sys.stderr)
        return 1
    return 0


def main():
    args = parse()
    if os.environ.get("LIME_BENCH_WATCHDOG"):  # debugging: every thread's stack, then exit
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["LIME_BENCH_WATCHDOG"]), exit=True)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}")
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and ndev < world:
        sys.exit(f"bench.py: RCCL needs one GPU per rank ({world} ranks, {ndev} GPUs); "
                 "--dist-backend gloo rehearses the sharded path with ranks sharing a GPU")
    # one rank per GPU; --dist-backend gloo lets several ranks share one GPU
    # (rehearsal of the multi-GPU path on a 1-GPU box, rows staged on the host)
    gpu = local % max(ndev, 1)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    comm_dev = None  # RCCL: device buffers
    args.sharded_step = world > 1 or (args.sharded and args.workload == "c2")
    if args.sharded_step and world == 1:  # a one-rank group (--sharded)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if args.sharded_step:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
            comm_dev = torch.device("cpu")

    import lime_amd
    from lime_amd import synth

    ctx = lime_amd.Context(dev.index)
    # one non-default stream shared by torch and the engine: the HIP events
    # below are recorded on the stream the kernels are launched on, and the
    # collectives are stream-ordered with the engine's kernels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    space = lime_amd.Space(list(synth.HG38.keys()), list(synth.HG38.values()))

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def measure(step, steps, warmup):
        """warmup untimed steps, then `steps` timed ones bracketed by a
        barrier + device sync; the max over ranks"""
        for _ in range(warmup):
            step(False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            step(i == steps - 1)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64, device=comm_dev or dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        return dt

    benches = {"c2": bench_c2, "c5": bench_c5, "c3": bench_c3, "sub": bench_sub}
    step, finish = benches[args.workload](args, ctx, space, dev, world, rank, comm_dev, ev)
    line = finish(measure(step, args.steps, args.warmup))
    if args.workload == "c2" and not args.no_ops:
        # the other operators north_star names, short lines at the same N
        # (the driver's scaling runs record them beside the metric)
        finish.release()
        ops = {}
        for name, fn in (("merge_side_c3", bench_c3), ("subtract_1b", bench_sub)):
            st, fi = fn(args, ctx, space, dev, world, rank, comm_dev, ev, brief=True)
            ops[name] = fi(measure(st, args.ops_steps, 1))
            fi.release()
        line["operators"] = ops
    line.setdefault("config", {}).update(
        {"world_size": world, "dist_backend": args.dist_backend if args.sharded_step else None,
         "sharded_step": bool(args.sharded_step),
         "launcher": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
         else ("bench.py --gpus N (own ranks)" if world > 1 else None)})
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if args.sharded_step:
        dist.destroy_process_group()


def bench_c2(args, ctx, space, dev, world, rank, comm_dev, ev):
    import torch
    n = args.rows or 100_000_000
    seed_a, seed_b = 0xA, 0xB
    # this rank's slice of the one C2 input (all of it at N = 1)
    first, last = rank * n // world, (rank + 1) * n // world
    m = last - first

    def gen(seed):
        c = torch.empty(m, dtype=torch.int32, device=dev)
        s = torch.empty(m, dtype=torch.int32, device=dev)
        e = torch.empty(m, dtype=torch.int32, device=dev)
        ctx.synth_uniform_rows(space, first, m, seed, 50, 5000, c.data_ptr(), s.data_ptr(),
                               e.data_ptr())
        return c, s, e
    A_in, B_in = gen(seed_a), gen(seed_b)
    chunk = args.chunk if world == 1 else min(args.chunk, max(1, 4 * (1 << 31) // world))
    buf = torch.empty((chunk, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    fills = []  # (start event, end event, pairs of the launch, pairs of the plan)
    state = {"phases": None, "npairs": 0, "nruns": 0, "halo": (0, 0), "routed": 0}

    def fill_all(plan):
        for f in range(0, plan.n, chunk):
            k = min(chunk, plan.n - f)
            e0 = ev()
            plan.fill_device(f, k, buf.data_ptr())
            fills.append((e0, ev(), k, plan.n))

    shard = None
    if args.sharded_step:
        from lime_amd.sharded import ShardStep
        shard = ShardStep(ctx, space, comm_device=comm_dev, shared_stream=True)
        # count-balanced shard bounds from samples of both inputs, once
        shard.plan_splits([(m, A_in[0].data_ptr(), A_in[1].data_ptr()),
                           (m, B_in[0].data_ptr(), B_in[1].data_ptr())])

    def step(last_step):
        t = [ev()] if last_step else None
        if shard is not None:
            A = shard.load(m, *(x.data_ptr() for x in A_in), row_base=first)
            B = shard.load(m, *(x.data_ptr() for x in B_in), row_base=first)
            if t is not None:
                t.append(ev())
            out = shard.run(A, B, on_pairs=fill_all)
            for h in (out["merge_a"], out["merge_b"], A, B):
                h.close()
            if t is not None:
                t.append(ev())
                state["phases"] = t
                state["halo"] = out["halo"]
            state["npairs"], state["nruns"] = out["pairs"], out["runs_a"] + out["runs_b"]
            return
        A = ctx.set_from_device(space, m, *(x.data_ptr() for x in A_in))
        B = ctx.set_from_device(space, m, *(x.data_ptr() for x in B_in))
        if t is not None:
            t.append(ev())
        plan = ctx.intersect(A, B)
        if t is not None:
            t.append(ev())
        fill_all(plan)
        if t is not None:
            t.append(ev())
        ma, mb = ctx.merge(A), ctx.merge(B)
        if t is not None:
            t.append(ev())
            state["phases"] = t
        state["npairs"], state["nruns"] = plan.n, ma.n + mb.n
        for h in (plan, ma, mb, A, B):
            h.close()

    def finish(dt):
        import torch.distributed as dist
        ms = dt / args.steps * 1e3
        value = 2 * n / (dt / args.steps)
        timed = fills[-args.steps * max(1, -(-state["npairs"] // chunk)):] if fills else []
        fill_ms = [a.elapsed_time(b) for a, b, _, _ in timed]
        # algorithmic bytes per launch: 16 B per pair written + 20 B per owner
        # row consumed (lo, count, start, end, row), prorated to the launch
        own = 2 * m
        fill_bytes = [16 * k + 20 * own * k / tot for _, _, k, tot in timed]
        avg_ms = sum(fill_ms) / max(len(fill_ms), 1)
        avg_b = sum(fill_bytes) / max(len(fill_bytes), 1)
        achieved = avg_b / (avg_ms * 1e-3) / 1e9 if avg_ms else 0.0
        p = state["phases"]
        if shard is not None:
            breakdown = {"route_sort_ms": p[0].elapsed_time(p[1]),
                         "merge_halo_count_fill_carry_ms": p[1].elapsed_time(p[2]),
                         "fill_ms": sum(fill_ms[-max(1, -(-state["npairs"] // chunk)):]),
                         "halo_rows": list(state["halo"]), "rows_routed_in": shard.routed}
        else:
            breakdown = {"sort_ms": p[0].elapsed_time(p[1]), "count_ms": p[1].elapsed_time(p[2]),
                         "fill_ms": p[2].elapsed_time(p[3]), "merge_ms": p[3].elapsed_time(p[4])}
        # the sort stage against its own roofline (24 B per
        # row algorithmic -- read 12, write 12), both sets
        sort_roof = None
        if world == 1 and breakdown.get("sort_ms"):
            sb = 24 * 2 * n
            sa = sb / (breakdown["sort_ms"] * 1e-3) / 1e9
            sort_roof = {"bound": "hbm", "achieved": sa, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": sa / HBM_PEAK_GBS, "alg_bytes": sb,
                         "kernels": "k_prep + 2 digit passes + k_local_small (bucketed sort)"}
        npairs, nruns = state["npairs"], state["nruns"]
        if world > 1:
            tt = torch.tensor([npairs, nruns], dtype=torch.int64, device=comm_dev or dev)
            dist.all_reduce(tt)
            npairs, nruns = (int(x) for x in tt.tolist())
        traffic, tsrc = pmc_traffic("pmc_c2.json", "hbm_bytes_per_launch", world)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_scale, n)
        return {
            "metric": "intervals/sec for pairwise intersect+merge at 1/2/4/8 GPUs; "
                      "% of HBM peak GB/s",
            "value": value, "unit": "intervals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (counter-based splitmix64, seeds 0xA/0xB; rank r generates "
                    "rows [r n/N, (r+1) n/N) of the one input)",
            "config": {"workload": "C2: sort + intersect + merge(A), merge(B); 2 x 1e8 "
                                   "intervals, uniform over hg38, len U[50,5000]"
                                   + (", one genome range-sharded over the ranks"
                                      if world > 1 else ""),
                       "rows_per_set": n, "pairs_per_step": npairs, "runs_per_step": nruns,
                       "output_chunk_pairs": chunk,
                       "parallelism": f"range-shard x{world}" if world > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": tsrc,
                         "kernel": "k_fill<1, false, false>", "avg_launch_ms": avg_ms,
                         "alg_bytes_per_launch": avg_b, "launches": len(timed)},
            "breakdown_ms": breakdown,
            "sort_roofline": sort_roof,
            "cpu_baseline": cpu,
        }

    def release():  # the output buffer and inputs, before other workloads run
        nonlocal buf, A_in, B_in
        buf = A_in = B_in = None
        torch.cuda.empty_cache()
    finish.release = release
    return step, finish


def bench_c5(args, ctx, space, dev, world, rank, comm_dev, ev):
    import torch

    from lime_amd.sharded import ShardedAnd
    k = 8
    per = args.rows or 125_000_000
    first, last = rank * per // world, (rank + 1) * per // world
    m = last - first
    ins = []
    for i in range(k):
        c = torch.empty(m, dtype=torch.int32, device=dev)
        s = torch.empty(m, dtype=torch.int32, device=dev)
        e = torch.empty(m, dtype=torch.int32, device=dev)
        ctx.synth_uniform_rows(space, first, m, 0x50 + i, 10, 40, c.data_ptr(), s.data_ptr(),
                               e.data_ptr())
        ins.append((c, s, e))
    torch.cuda.synchronize(dev)
    op = ShardedAnd(ctx, space, comm_device=comm_dev, shared_stream=True)
    if world > 1:  # count-balanced shard windows from samples of every set, once
        op.plan_splits([(m, X[0].data_ptr(), X[1].data_ptr(), X[2].data_ptr()) for X in ins])
    state = {"t": None, "runs": 0}

    def step(last_step):
        t0 = ev() if last_step else None
        out = op.run([(m, *(x.data_ptr() for x in X)) for X in ins])
        if last_step:
            state["t"] = (t0, ev())
        state["runs"] = out["runs_total"]
        out["result"].close()

    def finish(dt):
        ms = dt / args.steps * 1e3
        G = int(sum(synth_lengths()))
        W = (space.span + 63) // 64 * 8
        alg = 12 * k * per + k * W  # rows read once + k bitsets (G/8 each)
        achieved = alg / world / (ms * 1e-3) / 1e9
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = c5_cpu_baseline(100, per)
        traffic, tsrc = pmc_traffic("pmc_c5.json", "hbm_bytes_per_step", world)
        return {
            "metric": "intervals/sec for 8-way intersection (BASELINE C5); % of HBM peak GB/s",
            "value": k * per / (dt / args.steps), "unit": "intervals/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (counter-based splitmix64, seeds 0x50..0x57; rank r generates "
                    "rows [r n/N, (r+1) n/N) of every set)",
            "config": {"workload": f"C5: {k}-way intersection, {k} x {per} rows, len U[10,40], "
                                   "hg38, bit-per-base path" +
                                   (", range-sharded with clipped rows" if world > 1 else ""),
                       "sets": k, "rows_per_set": per, "runs_per_step": state["runs"],
                       "genome_bases": G,
                       "parallelism": f"range-shard x{world}" if world > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": tsrc,
                         "kernel": "whole C5 step (route, bin, paint, AND, extract) per GPU",
                         "alg_bytes_per_step_per_gpu": alg / world,
                         "step_ms_hip_events": state["t"][0].elapsed_time(state["t"][1])},
            "cpu_baseline": cpu,
        }
    return step, finish


def pmc_traffic(name, field, world):
    """HBM bytes (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, tools/pmc_json.py) of
    the same command, from a profile committed under profiles/, with where it
    came from (file, commit, command, kernel); (None, None) without one or at
    N > 1 (the profiles are single-GPU runs)"""
    p = os.path.join(ROOT, "profiles", name)
    if world != 1 or not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    src = dict(d.get("provenance", {}))
    src["file"] = os.path.join("profiles", name)
    if "key_kernel" in d:
        src["kernel"] = d["key_kernel"]
    return d.get(field), src


def _count_all(x, world, comm_dev, dev):
    """a per-rank count summed over the ranks"""
    import torch
    import torch.distributed as dist
    if world == 1:
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=comm_dev or dev)
    dist.all_reduce(t)
    return int(t.item())


def bench_c3(args, ctx, space, dev, world, rank, comm_dev, ev, brief=False):
    """north_star's merge side on C3's input (5e8 ChIP-seq-like pile-up rows:
    2e6 centres, N(0,150) offsets, len U[150,600], seed 0xC): sort, merge with
    every row's run id and the complement's gaps (Merge.scala:34-36,
    Complement.scala:131-134).  N > 1: the rows range-sharded, the merge
    carried across shards (one all_gather), global run ids, the sharded
    complement from the carry."""
    import torch
    n = args.rows if (args.rows and not brief) else 500_000_000
    first, last = rank * n // world, (rank + 1) * n // world
    m = last - first
    cols = [torch.empty(m, dtype=torch.int32, device=dev) for _ in range(3)]
    ctx.synth_pileup_rows(space, first, m, 0xC, 2_000_000, 150, 150, 600,
                          *(c.data_ptr() for c in cols))
    torch.cuda.synchronize(dev)
    shard = None
    if world > 1:
        from lime_amd.sharded import ShardStep
        shard = ShardStep(ctx, space, comm_device=comm_dev, shared_stream=True)
        shard.plan_splits([(m, cols[0].data_ptr(), cols[1].data_ptr())])
    state = {"runs": 0, "gaps": 0, "t": None}

    def step(last_step):
        t0 = ev() if last_step else None
        if shard is not None:
            S = shard.load(m, *(c.data_ptr() for c in cols), row_base=first)
            mg = shard.merge(S)
            _, ids = shard.global_run_ids(mg, S.n)
            gaps = shard.complement(S, mg)
            runs, ng = mg["runs"], gaps.n
            for h in (gaps, mg["result"], S):
                h.close()
            del ids
        else:
            S = ctx.set_from_device(space, m, *(c.data_ptr() for c in cols))
            mg = ctx.merge(S)
            # the complement from the merge's runs (as the sharded path:
            # one merge scan per step, Complement.scala's gaps of its runs)
            k = mg.n
            rgs = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
            rge = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
            if k:
                mg.copy_rows_device(0, k, rgs.data_ptr(), rge.data_ptr())
            gaps = ctx.complement_runs(space, k, rgs.data_ptr(), rge.data_ptr())
            runs, ng = mg.n, gaps.n
            for h in (gaps, mg, S):
                h.close()
            del rgs, rge
        if last_step:
            state["t"] = (t0, ev())
        state["runs"], state["gaps"] = runs, ng

    def finish(dt):
        steps = args.ops_steps if brief else args.steps
        ms = dt / steps * 1e3
        runs = _count_all(state["runs"], world, comm_dev, dev)
        gaps = _count_all(state["gaps"], world, comm_dev, dev)
        # per row: sort 24 B, merge 8 B read + 4 B run id; 8 B per run and gap
        alg = 36 * n + 8 * (runs + gaps)
        achieved = alg / world / (ms * 1e-3) / 1e9
        out = {"metric": "intervals/sec, merge side (sort + merge + run ids + complement) of "
                         "BASELINE C3", "value": n / (dt / steps), "unit": "intervals/s",
               "n_gpus": world, "steps": steps, "ms_per_step": ms, "higher_is_better": True,
               "scaling": "strong", "rows": n, "runs": runs, "gaps": gaps,
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                            "kernel": "whole step per GPU",
                            "alg_bytes_per_step_per_gpu": alg / world}}
        if not brief:
            out.update({"warmup": args.warmup, "vs_baseline": None, "dtype": "u32",
                        "data": "synthetic (counter-based splitmix64 pile-ups, seed 0xC; rank r "
                                "generates rows [r n/N, (r+1) n/N) of the one input)",
                        "config": {"workload": "C3: merge side of 5e8 pile-up intervals "
                                               "(2e6 centres, N(0,150), len U[150,600]), hg38"
                                               + (", range-sharded" if world > 1 else ""),
                                   "parallelism": f"range-shard x{world}" if world > 1
                                   else "1 GPU"}})
        return out

    def release():
        cols.clear()
        torch.cuda.empty_cache()
    finish.release = release
    return step, finish


def bench_sub(args, ctx, space, dev, world, rank, comm_dev, ev, brief=False):
    """north_star's difference on its 1B-interval sets: DistributedSubtract
    (lime mode, Subtract.scala:78-116) of 2 x 5e8 rows uniform over hg38, len
    U[10,40] (seeds 0x1A / 0x1C: the pairwise side of tests/test_gpu_scale.py
    and tools/bench_extra.py b1_pair): sort both, A minus B, every remnant
    materialised (~7.4e7 records: C2's deep inputs leave only 16).  N > 1:
    both sets range-sharded, B with its left and right halos (rows of other
    shards reaching into the shard), outputs disjoint by A row."""
    import torch
    n = args.rows if (args.rows and not brief) else 500_000_000
    first, last = rank * n // world, (rank + 1) * n // world
    m = last - first

    def gen(seed):
        cols = [torch.empty(m, dtype=torch.int32, device=dev) for _ in range(3)]
        ctx.synth_uniform_rows(space, first, m, seed, 10, 40, *(c.data_ptr() for c in cols))
        return cols
    A_in, B_in = gen(0x1A), gen(0x1C)
    torch.cuda.synchronize(dev)
    shard = None
    if world > 1:
        from lime_amd.sharded import ShardStep
        shard = ShardStep(ctx, space, comm_device=comm_dev, shared_stream=True)
        shard.plan_splits([(m, A_in[0].data_ptr(), A_in[1].data_ptr()),
                           (m, B_in[0].data_ptr(), B_in[1].data_ptr())])
    state = {"records": 0}

    def step(last_step):
        if shard is not None:
            A = shard.load(m, *(c.data_ptr() for c in A_in), row_base=first)
            B = shard.load(m, *(c.data_ptr() for c in B_in), row_base=first)
            res, _, Be = shard.subtract(A, B)
            hs = (res, Be, A, B) if Be is not B else (res, A, B)
        else:
            A = ctx.set_from_device(space, m, *(c.data_ptr() for c in A_in))
            B = ctx.set_from_device(space, m, *(c.data_ptr() for c in B_in))
            res = ctx.subtract(A, B)
            hs = (res, A, B)
        state["records"] = res.n
        for h in hs:
            h.close()

    def finish(dt):
        steps = args.ops_steps if brief else args.steps
        ms = dt / steps * 1e3
        rec = _count_all(state["records"], world, comm_dev, dev)
        # sort 24 B per row of both sets; A rows read 12 B, B 16 B (rows and
        # prefix max); 16 B per record
        alg = 48 * n + 28 * n + 16 * rec
        achieved = alg / world / (ms * 1e-3) / 1e9
        out = {"metric": "intervals/sec, DistributedSubtract (lime mode) of the 1B-interval "
                         "sets (2 x 5e8)", "value": 2 * n / (dt / steps), "unit": "intervals/s",
               "n_gpus": world, "steps": steps, "ms_per_step": ms, "higher_is_better": True,
               "scaling": "strong", "rows_per_set": n, "records": rec,
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                            "kernel": "whole step per GPU",
                            "alg_bytes_per_step_per_gpu": alg / world}}
        if not brief:
            out.update({"warmup": args.warmup, "vs_baseline": None, "dtype": "u32",
                        "data": "synthetic (counter-based splitmix64, seeds 0x1A/0x1C; rank r "
                                "generates rows [r n/N, (r+1) n/N) of each input)",
                        "config": {"workload": "subtract (lime mode) of 2 x 5e8 intervals, "
                                               "uniform over hg38, len U[10,40]"
                                               + (", range-sharded with halos" if world > 1
                                                  else ""),
                                   "parallelism": f"range-shard x{world}" if world > 1
                                   else "1 GPU"}})
        return out

    def release():
        A_in.clear()
        B_in.clear()
        torch.cuda.empty_cache()
    finish.release = release
    return step, finish


def synth_lengths():
    from lime_amd import synth
    return list(synth.HG38.values())


if __name__ == "__main__":
    main()
