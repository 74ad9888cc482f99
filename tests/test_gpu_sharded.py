"""Range-sharded engine paths on the GPU: 1-4 ranks sharing the one MI355X
of the test box (gloo carries the rows, staged through the host), one genome
cut into coordinate ranges so that intervals DO cross shard boundaries.
Every rank starts from an arbitrary slice of the unsorted input (the device
router moves rows to their owner shards).  The union of the shards' owned
pairs and carried merge runs (C2's path), and the gathered k-way AND runs
(C5's path), must equal the single-shard oracle result."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

LENS = [300_000, 200_000, 250_000]
NAMES = ["c0", "c1", "c2"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows():
    from lime_amd import synth
    A = synth.uniform(LENS, 20000, 0x11, 10, 6000)
    B = synth.uniform(LENS, 15000, 0x22, 10, 9000)
    return A, B


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    # a failing rank must not leave its peers blocked in a collective
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        import lime_amd
        from lime_amd import dist as ld
        from lime_amd.sharded import ShardStep
        ctx = lime_amd.Context(0)
        sp = lime_amd.Space(NAMES, LENS)
        off = sp.offsets
        A, B = _rows()
        step = ShardStep(ctx, sp, comm_device=torch.device("cpu"))

        def load(X):
            # this rank's arbitrary slice of the UNSORTED input, on the device;
            # load() routes it to the owner shards (row ids stay global)
            n = len(X[0])
            f, l = rank * n // world, (rank + 1) * n // world
            t = [torch.from_numpy(np.ascontiguousarray(x[f:l]).astype(np.int32)).cuda()
                 for x in X]
            torch.cuda.synchronize()
            S = step.load(l - f, *(x.data_ptr() for x in t), row_base=f)
            h = S.to_host()
            g = off[h["contig"]] + h["start"]
            assert ((g >= step.splits[rank]) & (g < step.splits[rank + 1])).all()
            return S
        Aset, Bset = load(A), load(B)
        got = []

        def on_pairs(plan):
            p = plan.fill_host()
            got.extend(zip(p["a_row"].tolist(), p["b_row"].tolist(), p["start"].tolist(),
                           p["end"].tolist()))
        out = step.run(Aset, Bset, on_pairs=on_pairs)
        # merged runs after the carry, in local coordinates
        runs = []
        for key, res in (("a", out["merge_a"]), ("b", out["merge_b"])):
            d, e = out["drop"][0 if key == "a" else 1], out["extend"][0 if key == "a" else 1]
            h = res.to_host()
            st, en, ct = list(h["start"]), list(h["end"]), list(h["contig"])
            st, en, ct = st[d:], en[d:], ct[d:]
            if e is not None and st:
                en[-1] = e - off[ct[-1]]
            runs.append(list(zip(ct, st, en)))
        q.put((rank, got, runs, out["halo"], step.routed))
        ctx.close()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_engine_matches_single_shard(world):
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[1] == "error"]
    assert not errs, errs[0]
    for p in ps:
        assert p.exitcode == 0
    A, B = _rows()
    exp = oracle.intersect(A, B)
    want = sorted(zip(exp["a_row"].tolist(), exp["b_row"].tolist(), exp["start"].tolist(),
                      exp["end"].tolist()))
    got = sorted(sum((r[1] for r in res), []))
    assert got == want
    assert sum(r[3][0] + r[3][1] for r in res) > 0  # boundary rows really moved (halo)
    assert sum(r[4] for r in res) > 0                 # and the input was routed
    for k, X in ((0, A), (1, B)):
        m = oracle.merge(X)
        runs = sum((r[2][k] for r in res), [])
        assert [tuple(map(int, t)) for t in runs] == \
            list(zip(m["contig"].tolist(), m["start"].tolist(), m["end"].tolist()))


# ------------------------------------------------------------ sharded C5
C5_LENS = [3_000_000, 2_000_000, 2_500_000]
C5_K, C5_N = 4, 120_000  # rows per set (all ranks together), len U[10, 400]


def _c5_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        import lime_amd
        from lime_amd.sharded import ShardedAnd
        ctx = lime_amd.Context(0)
        sp = lime_amd.Space(NAMES, C5_LENS)
        # this rank's slice of every set: rows [first, first + m) of the
        # counter-based generator, unsorted, on the device
        first, last = rank * C5_N // world, (rank + 1) * C5_N // world
        m = last - first
        inputs, keep = [], []
        for i in range(C5_K):
            c = torch.empty(m, dtype=torch.int32, device="cuda")
            s = torch.empty(m, dtype=torch.int32, device="cuda")
            e = torch.empty(m, dtype=torch.int32, device="cuda")
            ctx.synth_uniform_rows(sp, first, m, 0x70 + i, 10, 400, c.data_ptr(), s.data_ptr(),
                                   e.data_ptr())
            keep.append((c, s, e))
            inputs.append((m, c.data_ptr(), s.data_ptr(), e.data_ptr()))
        ctx.synchronize()
        step = ShardedAnd(ctx, sp, comm_device=torch.device("cpu"))
        out = step.run(inputs, gather=True)
        q.put((rank, out["runs"].numpy().tolist(), out["runs_total"], step.moved,
               [int(x) for x in sp.offsets]))
        out["result"].close()
        ctx.close()
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_c5_matches_single_shard_oracle(world):
    # BASELINE C5's sharded path (route + clip + all_to_all + windowed
    # bitsets + AND + boundary carry + allgatherv) with `world` ranks sharing
    # the GPU (gloo), against the oracle fold of intersect over the merged
    # operands (coalesced book-ended runs)
    from lime_amd import synth
    from oracle import oracle
    from tests.test_gpu_configs import coalesce, fold_and
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_c5_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[1] == "error"]
    assert not errs, errs[0]
    for p in ps:
        assert p.exitcode == 0
    off = np.array(res[0][4])
    merged = []
    for i in range(C5_K):
        X = synth.uniform(C5_LENS, C5_N, 0x70 + i, 10, 400)
        merged.append(oracle.merge_mt(len(C5_LENS), X))
    exp = fold_and(len(C5_LENS), merged)
    want = coalesce(exp["contig"], exp["start"], exp["end"])
    for r in res:
        runs = np.array(r[1], dtype=np.int64).reshape(-1, 2)
        # global -> (contig, local)
        c = np.searchsorted(off, runs[:, 0], side="right") - 1
        got = coalesce(c, runs[:, 0] - off[c], runs[:, 1] - off[c])
        for x, y in zip(got, want):
            assert np.array_equal(x, y)
        assert r[2] == len(runs)
    if world > 1:
        assert sum(r[3] for r in res) > 0  # rows really moved between shards


# ------------------------------------------- sharded subtract and C4 ops
def _c4_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        import lime_amd
        from lime_amd import SUBTRACT_LIME, SUBTRACT_SET
        from lime_amd.sharded import ShardedBitset, ShardStep
        ctx = lime_amd.Context(0)
        sp = lime_amd.Space(NAMES, LENS)
        A, B = _rows()
        dev_rows = []
        for X in (A, B):
            n = len(X[0])
            f, l = rank * n // world, (rank + 1) * n // world
            t = [torch.from_numpy(np.ascontiguousarray(x[f:l]).astype(np.int32)).cuda()
                 for x in X]
            dev_rows.append((f, l - f, t))
        torch.cuda.synchronize()
        out = {}
        # subtract (interval path): own A rows against left + own + right B
        step = ShardStep(ctx, sp, comm_device=torch.device("cpu"))
        S = [step.load(m, *(x.data_ptr() for x in t), row_base=f) for f, m, t in dev_rows]
        for mode in (SUBTRACT_LIME, SUBTRACT_SET):
            for thr in (0, 25):
                res, halo, Be = step.subtract(S[0], S[1], thr, mode)
                h = res.to_host()
                out[("sub", mode, thr)] = (list(zip(h["contig"].tolist(), h["start"].tolist(),
                                                    h["end"].tolist(), h["a_row"].tolist(),
                                                    h["b_row"].tolist())), halo)
                res.close()
                if Be is not S[1]:
                    Be.close()
        # complement (NOT) and difference (AND-NOT) on shard windows
        bits = ShardedBitset(ctx, sp, comm_device=torch.device("cpu"))
        inp = [(m, *(x.data_ptr() for x in t)) for f, m, t in dev_rows]
        for op, args in (("not", inp[:1]), ("andnot", inp)):
            r = bits.run(args, gather=True, op=op)
            out[op] = r["runs"].numpy().tolist()
            r["result"].close()
        q.put((rank, out, [int(x) for x in sp.offsets]))
        ctx.close()
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_subtract_and_c4_ops(world):
    # sharded subtract (both modes, two thresholds) == the oracle on all rows;
    # sharded complement / difference on shard windows == the oracle's
    # complement / set-mode subtract of merged runs (per base, coalesced)
    from lime_amd import SUBTRACT_LIME, SUBTRACT_SET
    from oracle import oracle
    from tests.test_gpu_configs import coalesce
    from tests.util import as_sorted_tuples
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[1] == "error"]
    assert not errs, errs[0]
    A, B = _rows()
    for mode in (SUBTRACT_LIME, SUBTRACT_SET):
        for thr in (0, 25):
            got = sorted(sum((r[1][("sub", mode, thr)][0] for r in res), []))
            assert got == as_sorted_tuples(oracle.subtract(A, B, thr, mode))
    assert sum(r[1][("sub", SUBTRACT_LIME, 0)][1][0] for r in res) > 0  # left halo moved
    off = np.array(res[0][2])

    def local(runs):
        runs = np.array(runs, dtype=np.int64).reshape(-1, 2)
        c = np.searchsorted(off, runs[:, 0], side="right") - 1
        return coalesce(c, runs[:, 0] - off[c], runs[:, 1] - off[c])
    comp = oracle.complement(A, LENS)
    ma, mb = oracle.merge(A), oracle.merge(B)
    diff = oracle.subtract((ma["contig"], ma["start"], ma["end"]),
                           (mb["contig"], mb["start"], mb["end"]), 0, oracle.SUB_SET)
    for r in res:
        for op, exp in (("not", comp), ("andnot", diff)):
            got = local(r[1][op])
            want = coalesce(exp["contig"], exp["start"], exp["end"])
            for x, y in zip(got, want):
                assert np.array_equal(x, y), op


# ------------------- sharded complement, global run ids, stranded sets
def _strand_rows(bounds=None):
    """A (with strands 1 / 2, zero-width rows, rows on the shard bounds:
    `bounds`, by default the 2- and 3-way even splits) and B, contig-local"""
    from lime_amd import Space, synth
    from lime_amd import dist as ld
    A = [np.asarray(x) for x in synth.uniform(LENS, 12000, 0x33, 0, 4000)]
    B = [np.asarray(x) for x in synth.uniform(LENS, 9000, 0x44, 10, 5000)]
    sp_off = np.concatenate([[0], np.cumsum(np.array(LENS) + 1)])
    if bounds is None:
        bounds = [b for w in (2, 3) for b in ld.even_splits(int(sp_off[-1]), w)[1:-1]]
    extra = []
    for b in bounds:
        c = int(np.searchsorted(sp_off, b, side="right") - 1)
        s = int(b - sp_off[c])
        if 60 < s < LENS[c] - 60:
            extra += [(c, s, s), (c, s - 50, s), (c, s, s + 40), (c, s - 5, s + 5)]
    for i, col in enumerate(zip(*extra)):
        A[i] = np.concatenate([A[i], np.array(col, A[i].dtype)])
    rng = np.random.default_rng(5)
    sa = rng.integers(1, 3, len(A[0])).astype(np.int8)
    sb = rng.integers(1, 3, len(B[0])).astype(np.int8)
    return A, B, sa, sb


def _strand_worker(rank, world, port, q, mode="even"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        import lime_amd
        from lime_amd import dist as ld
        from lime_amd.sharded import ShardStep
        ctx = lime_amd.Context(0)
        sp = lime_amd.Space(NAMES, LENS)
        off = sp.offsets
        out = {}

        def dev(X, st=None):
            n = len(X[0])
            f, l = rank * n // world, (rank + 1) * n // world
            t = [torch.from_numpy(np.ascontiguousarray(x[f:l]).astype(np.int32)).cuda()
                 for x in X]
            s8 = torch.from_numpy(np.ascontiguousarray(st[f:l])).cuda() if st is not None \
                else None
            torch.cuda.synchronize()
            return l - f, t, s8, f
        if mode == "even":
            # (_strand_rows puts rows on exactly these shard bounds)
            A, B, sa, sb = _strand_rows()
            splits = ld.even_splits(int(sp.offsets[-1]), world)
        else:
            # count-balanced bounds sampled from both inputs (plan_splits),
            # then rows placed exactly on those bounds
            A0, B0, _, _ = _strand_rows([])
            (na, ta, _, _), (nb, tb, _, _) = dev(A0), dev(B0)
            planner = ShardStep(ctx, sp, comm_device=torch.device("cpu"))
            splits = planner.plan_splits([(na, ta[0].data_ptr(), ta[1].data_ptr()),
                                          (nb, tb[0].data_ptr(), tb[1].data_ptr())])
            assert splits != ld.even_splits(int(sp.offsets[-1]), world)
            A, B, sa, sb = _strand_rows(splits[1:-1])
        out["splits"] = list(splits)
        step = ShardStep(ctx, sp, splits=splits, comm_device=torch.device("cpu"))
        # plain: merge run ids + the shard's complement gaps
        n, t, _, f = dev(A)
        S = step.load(n, *(x.data_ptr() for x in t), row_base=f)
        m = step.merge(S)
        rows, gid = step.global_run_ids(m, S.n)
        out["ids"] = list(zip(rows.cpu().tolist(), gid.cpu().tolist()))
        m["result"].close()
        comp = step.complement(S).to_host()
        lo, hi = step.splits[rank], step.splits[rank + 1]
        g = off[comp["contig"]] + comp["start"]
        assert ((g >= lo) & (g < hi)).all()
        out["comp"] = list(zip(comp["contig"].tolist(), comp["start"].tolist(),
                               comp["end"].tolist()))
        # stranded: merge (runs break at strand changes) + its run ids
        n, t, s8, f = dev(A, sa)
        SS = step.load(n, *(x.data_ptr() for x in t), row_base=f, d_strand=s8.data_ptr())
        m = step.merge(SS, stranded=True)
        h = m["result"].to_host()
        st_ = m["result"].run_strands(0, m["result"].n)
        k = m["drop"]
        runs = [list(x) for x in zip(h["contig"].tolist(), h["start"].tolist(),
                                     h["end"].tolist(), st_.tolist())][k:]
        if m["ext"] is not None and runs:
            runs[-1][2] = m["ext"] - int(off[runs[-1][0]])
        out["sruns"] = [tuple(r) for r in runs]
        rows, gid = step.global_run_ids(m, SS.n)
        out["sids"] = list(zip(rows.cpu().tolist(), gid.cpu().tolist()))
        # stranded pairwise: strand groups of A and B, intersect per group
        na, ta, s8a, fa = dev(A, sa)
        nb, tb, s8b, fb = dev(B, sb)
        GA = step.load_strand_groups(na, *(x.data_ptr() for x in ta), s8a.data_ptr(), fa)
        GB = step.load_strand_groups(nb, *(x.data_ptr() for x in tb), s8b.data_ptr(), fb)
        pairs = []
        for code in (1, 2):  # every rank runs every code (collectives line up)
            Ga = GA.get(code) or ctx.set_from_global(sp, 0, 0, 0, 0)
            Gb = GB.get(code) or ctx.set_from_global(sp, 0, 0, 0, 0)

            def on_pairs(plan):
                p = plan.fill_host()
                pairs.extend(zip(p["a_row"].tolist(), p["b_row"].tolist()))
            step.run(Ga, Gb, on_pairs=on_pairs)
        out["spairs"] = pairs
        q.put((rank, out))
        ctx.close()
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "even"), (3, "even"), (3, "sampled")])
def test_sharded_complement_run_ids_strands(world, mode):
    # SURVEY.md 8(e) on the device: the shards' complement gaps, the global
    # run id of every row (plain and stranded merge) and stranded pairs equal
    # the single-shard oracle (Complement.scala:39-45,67-73,112-122;
    # SetTheory.scala:213-217,263-272; cli/Intersection.scala:45,48)
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_strand_worker, args=(r, world, port, q, mode))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[1]["error"] for r in res if "error" in r[1]]
    assert not errs, errs[0]
    A, B, sa, sb = _strand_rows(None if mode == "even" else res[0][1]["splits"][1:-1])
    m = oracle.merge(A)
    ids = dict(sum((r[1]["ids"] for r in res), []))
    assert [ids[i] for i in range(len(A[0]))] == m["run_of_row"].tolist()
    comp = oracle.complement(A, LENS)
    got = sorted(sum((r[1]["comp"] for r in res), []))
    assert got == list(zip(comp["contig"].tolist(), comp["start"].tolist(), comp["end"].tolist()))
    ms = oracle.merge((A[0], A[1], A[2], sa))
    runs = sum((r[1]["sruns"] for r in res), [])
    assert runs == list(zip(ms["contig"].tolist(), ms["start"].tolist(), ms["end"].tolist(),
                            ms["strand"].tolist()))
    ids = dict(sum((r[1]["sids"] for r in res), []))
    assert [ids[i] for i in range(len(A[0]))] == ms["run_of_row"].tolist()
    ix = oracle.intersect((A[0], A[1], A[2], sa), (B[0], B[1], B[2], sb))
    got = sorted(sum((r[1]["spairs"] for r in res), []))
    want = sorted(zip(ix["a_row"].tolist(), ix["b_row"].tolist()))
    if got != want:
        from collections import Counter
        g, w = Counter(got), Counter(want)
        extra, missing = list((g - w).items())[:5], list((w - g).items())[:5]
        info = [(p, [(int(X[0][i]), int(X[1][i]), int(X[2][i]), int(st[i]))
                     for X, st, i in ((A, sa, p[0][0]), (B, sb, p[0][1]))]) for p in extra + missing]
        raise AssertionError(f"{len(got)} vs {len(want)} pairs; extra {extra}; missing {missing}; "
                             f"rows {info}")


def _rccl_rounds_worker(port, q):
    # a one-rank RCCL group with the collectives forced on (no world-1
    # shortcut) and 64 MiB rounds: 1.2 GB of rows in 18 rounds, every row
    # back in place -- one all_to_all_single of 1.2 GB moves only its first
    # 600 MB on this image's RCCL (tools/rccl_probe.py --big)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                      WORLD_SIZE="1", LIME_A2A_FORCE="1", LIME_A2A_MAX_BYTES=str(64 << 20))
    import torch
    import torch.distributed as dist
    from lime_amd import dist as ld
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        n = 100_000_000
        buf = torch.randint(0, 1 << 30, (n, 3), dtype=torch.int32, device=dev)
        r, rc = ld.exchange_rows(buf, [n])
        ok_rows = rc == [n] and torch.equal(r, buf)
        del r
        small = [buf[:1000, :2].contiguous(), buf[1000:1500, :2].contiguous()]
        got = ld.exchange_sets_rows(small, [[1000], [500]])
        ok_sets = all(torch.equal(torch.cat(sl), x) and m == x.shape[0] and moved == 0
                      for (sl, m, moved), x in zip(got, small))
        q.put((bool(ok_rows), bool(ok_sets)))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_rounds_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rounds_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=150)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res == (True, True)


@pytest.mark.parametrize("nsh", [1, 5, 9, 64])
def test_route_rows_many_shards(nsh):
    # lime_route_rows / _interleaved against numpy on one process: every
    # piece at its destination in input order, clipped or not, 2- and
    # 3-word interleaved rows and the column form; misaligned inputs take
    # the scalar-load path (the write pass's counts go four destinations to
    # a block scan: nsh 5, 9, 64 cross those groups)
    import torch
    import lime_amd
    ctx = lime_amd.Context(0)
    sp = lime_amd.Space(NAMES, LENS)
    off = sp.offsets
    span = int(sp.span)
    rng = np.random.default_rng(1000 + nsh)
    n = 200_003
    c = rng.integers(0, len(LENS), n).astype(np.int32)
    L = np.array(LENS)[c]
    s = (rng.random(n) * (L - 1)).astype(np.int64)
    e = np.minimum(s + rng.integers(0, 40_000, n), L)
    g0 = off[c] + s
    g1 = off[c] + e
    cuts = np.sort(rng.choice(np.arange(1, span), nsh - 1, replace=False)) if nsh > 1 else []
    splits = [0] + [int(x) for x in cuts] + [span]
    dev = torch.device("cuda", 0)
    for shift in (0, 1):  # 1: inputs one element off 16-B alignment
        cols = [torch.from_numpy(np.concatenate([np.zeros(shift, x.dtype), x]).astype(np.int32))
                .to(dev)[shift:] for x in (c, s, e)]
        torch.cuda.synchronize()
        ptrs = [t.data_ptr() for t in cols]
        for clip in (False, True):
            sa = np.array(splits, np.int64)
            d0 = np.searchsorted(sa, g0, side="right") - 1
            wide = clip & (g1 > g0)
            d1 = np.where(wide, np.searchsorted(sa, g1 - 1, side="right") - 1, d0)
            per = d1 - d0 + 1
            rows = np.repeat(np.arange(n), per)
            dd = np.repeat(d0, per) + (np.arange(per.sum()) - np.repeat(np.cumsum(per) - per, per))
            a, b = g0[rows], g1[rows]
            if clip:
                a = np.maximum(a, sa[dd])
                b = np.where(wide[rows], np.minimum(b, sa[dd + 1]), b)
            order = np.argsort(dd, kind="stable")  # by destination, input order kept
            want = np.stack([a[order], b[order], 7 + rows[order]], 1).astype(np.int64)
            exp_cnt = np.bincount(dd, minlength=nsh).tolist()
            m = len(want)
            for k in (2, 3):
                buf = torch.empty((max(m, 1), k), dtype=torch.int32, device=dev)
                cnt = ctx.route_rows_interleaved(sp, n, *ptrs, splits, k, buf.data_ptr(),
                                                 clip=clip, cap=m, row_base=7)
                torch.cuda.synchronize()
                assert cnt == exp_cnt, (shift, clip, k)
                got = buf[:m].cpu().numpy().view(np.uint32).astype(np.int64)
                assert np.array_equal(got, want[:, :k]), (shift, clip, k)
            outs = [torch.empty(max(m, 1), dtype=torch.int32, device=dev) for _ in range(3)]
            cnt = ctx.route_rows(sp, n, *ptrs, splits, clip=clip, cap=m,
                                 d_gs=outs[0].data_ptr(), d_ge=outs[1].data_ptr(),
                                 d_row=outs[2].data_ptr(), row_base=7)
            torch.cuda.synchronize()
            got = np.stack([o[:m].cpu().numpy().view(np.uint32).astype(np.int64) for o in outs], 1)
            assert cnt == exp_cnt and np.array_equal(got, want)


def test_bench_sharded_step_matches_unsharded():
    # bench.py's C2 step through ShardStep in a one-rank RCCL group
    # (--sharded: route, exchange, global-row sort, carry all_gather, owned
    # pairs) reports the unsharded step's pair and run totals
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(*extra):
        cmd = [sys.executable, "bench.py", "--no-ops", "--no-cpu-baseline", "--steps", "1",
               "--warmup", "0", "--rows", "2000000", *extra]
        env = dict(os.environ)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
        return json.loads(line)
    plain, sharded = run(), run("--sharded")
    assert sharded["config"]["sharded_step"] and not plain["config"]["sharded_step"]
    for k in ("pairs_per_step", "runs_per_step"):
        assert sharded["config"][k] == plain["config"][k] > 0, k
