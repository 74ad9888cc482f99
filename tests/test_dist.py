"""Multi-process range sharding (lime_amd.dist) on the CPU with gloo.

World sizes 2 and 3, spawned processes, CPU tensors.  The data movement is
the product code; the per-shard compute is the oracle (these processes have
no GPU), and the union of shard outputs must equal the single-shard result,
whatever the shard count (the reference is shard-count dependent: Q1/Q2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lime_amd import dist as ld


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(seed, n, span, maxlen):
    rng = np.random.default_rng(seed)
    gs = rng.integers(0, span - maxlen, n)
    ge = gs + rng.integers(0, maxlen, n)
    return gs.astype(np.int64), ge.astype(np.int64)


def _owned_pairs(a, b):
    """oracle intersect of (A, B) rows given as (gs, ge, row) arrays, single
    contig in global coordinates; pair owner = smaller start (ties to a)."""
    from oracle import oracle
    A = (np.zeros(len(a[0]), np.int32), a[0], a[1])
    B = (np.zeros(len(b[0]), np.int32), b[0], b[1])
    r = oracle.intersect(A, B)
    ai, bi = r["a_row"], r["b_row"]
    return ai, bi, a[0][ai] <= b[0][bi]


def _worker(rank, world, port, q, splits_mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        from oracle import oracle
        span, n = 200_000, 3000
        gA, eA = _data(1, n, span, 900)
        gB, eB = _data(2, n, span, 2500)
        # every rank starts with a different arbitrary slice of the input
        sl = slice(rank * n // world, (rank + 1) * n // world)
        rowsA = np.arange(n)[sl]
        rowsB = np.arange(n)[sl]
        tA = [torch.from_numpy(x[sl].copy()) for x in (gA, eA)] + [torch.from_numpy(rowsA)]
        tB = [torch.from_numpy(x[sl].copy()) for x in (gB, eB)] + [torch.from_numpy(rowsB)]
        if splits_mode == "even":
            splits = ld.even_splits(span, world)
        else:
            splits = ld.sample_splits(torch.cat([tA[0], tB[0]]), span, world)
        A = ld.route_rows(*tA, splits)
        B = ld.route_rows(*tB, splits)
        assert all(((x >= splits[rank]) & (x < splits[rank + 1])).all() for x in (A[0], B[0]))

        def srt(s):
            o = torch.argsort(s[0] * 4 * n + s[2])  # by start, then row (deterministic)
            return tuple(x[o] for x in s)
        A, B = srt(A), srt(B)
        (hA, hB) = ld.right_halo([A, B])
        # own rows first, halo after (sorted: halo starts lie in later shards)
        ea = [torch.cat([A[i], hA[i]]).numpy() for i in range(3)]
        eb = [torch.cat([B[i], hB[i]]).numpy() for i in range(3)]
        na, nb = A[0].numel(), B[0].numel()
        ai, bi, a_owns = _owned_pairs(ea, eb)
        keep = np.where(a_owns, ai < na, bi < nb)
        pairs = sorted(zip(ea[2][ai[keep]].tolist(), eb[2][bi[keep]].tolist()))
        # merge with the one-step carry
        m = oracle.merge((np.zeros(na, np.int32), A[0].numpy(), A[1].numpy()))
        rs, re = torch.from_numpy(m["start"]), torch.from_numpy(m["end"])
        drop, new_end = ld.merge_carry(rs, re, k=2)  # tiny k exercises the regather
        rs, re = rs[drop:].clone(), re[drop:].clone()
        if new_end is not None and rs.numel():
            re[-1] = new_end
        runs = list(zip(rs.tolist(), re.tolist()))
        q.put((rank, pairs, runs, na, nb))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "even"), (3, "sample"), (4, "even")])
def test_sharded_intersect_and_merge(world, mode):
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    pairs = sorted(sum((r[1] for r in res), []))
    runs = sum((r[2] for r in res), [])
    assert sum(r[3] for r in res) == 3000 and sum(r[4] for r in res) == 3000
    span, n = 200_000, 3000
    gA, eA = _data(1, n, span, 900)
    gB, eB = _data(2, n, span, 2500)
    z = np.zeros(n, np.int32)
    full = oracle.intersect((z, gA, eA), (z, gB, eB))
    assert pairs == sorted(zip(full["a_row"].tolist(), full["b_row"].tolist()))
    assert len(pairs) == len(set(pairs))  # shard outputs are disjoint
    m = oracle.merge((z, gA, eA))
    assert runs == list(zip(m["start"].tolist(), m["end"].tolist()))


# ------------------------------------------- bitset sharding (C5 host logic)
def _runs_of(bits, lo):
    """runs of a 0/1 array as (global start, end)"""
    d = np.diff(np.concatenate([[0], bits.astype(np.int8), [0]]))
    s, e = np.flatnonzero(d == 1), np.flatnonzero(d == -1)
    return np.stack([s + lo, e + lo], axis=1).astype(np.int64)


def _and_sets(span, k, n, seed, maxlen):
    """k sets of n rows; every 50th row is long (up to 40 shard-widths of
    64), so runs cross and swallow whole shards"""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        g = rng.integers(0, span - 20 * maxlen, n)
        ln = rng.integers(0, maxlen, n)
        ln[::50] = rng.integers(maxlen, 20 * maxlen, len(ln[::50]))
        out.append((g, g + ln))
    return out


def _bits_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        span, k, n = 50_000, 3, 400
        sets = _and_sets(span, k, n, 7, 300)
        splits = ld.coord_splits(span, world, align=64)
        lo, hi = splits[rank], splits[rank + 1]
        acc = np.ones(hi - lo, bool)
        for g, e in sets:
            # this rank's slice of the rows, clipped and routed (the device
            # router's rule, restated), moved by the product exchange
            sl = slice(rank * n // world, (rank + 1) * n // world)
            pieces = [[] for _ in range(world)]
            for a, b in zip(g[sl], e[sl]):
                for r in range(world):
                    s_, e_ = max(a, splits[r]), min(b, splits[r + 1])
                    if e_ > s_:
                        pieces[r].append((s_, e_))
            counts = [len(p) for p in pieces]
            flat = [x for p in pieces for x in p] or [(0, 0)]
            gs = torch.tensor([x[0] for x in flat], dtype=torch.int32)
            ge = torch.tensor([x[1] for x in flat], dtype=torch.int32)
            (rgs, rge), rc = ld.exchange([gs, ge], counts)
            cov = np.zeros(hi - lo, bool)
            for a, b in zip(rgs.tolist(), rge.tolist()):
                assert lo <= a and b <= hi
                cov[a - lo:b - lo] = True
            acc &= cov
        runs = _runs_of(acc, lo)
        n_r = len(runs)
        fs, fe, le = (int(runs[0, 0]), int(runs[0, 1]), int(runs[-1, 1])) if n_r else (-1, -1, -1)
        drop, ext = ld.bitset_carry(n_r, fs, fe, le)
        mine = runs[drop:].copy()
        if ext is not None and len(mine):
            mine[-1, 1] = ext
        allr, _ = ld.allgatherv(torch.from_numpy(mine))
        q.put((rank, allr.numpy().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_bitset_and_carry(world):
    # shard-count invariance of the C5 boundary logic: rows clipped at shard
    # bounds, per-shard AND, book-ended runs re-joined by bitset_carry, the
    # emulated allgatherv == the unsharded per-base AND
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bits_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    span, k, n = 50_000, 3, 400
    acc = np.ones(span, bool)
    for g, e in _and_sets(span, k, n, 7, 300):
        cov = np.zeros(span, bool)
        for a, b in zip(g, e):
            cov[a:b] = True
        acc &= cov
    want = _runs_of(acc, 0).tolist()
    assert len(want) > 30
    for _, got in res:
        assert got == want  # every rank holds the whole ordered list


# ---------------- sharded merge run ids, complement, stranded carry (8(e))
_GENOME = [70_000, 55_000, 90_000]  # three contigs, bounds inside shards


def _offsets():
    off = [0]
    for L in _GENOME:
        off.append(off[-1] + L + 1)
    return off


def _to_local(g):
    off = np.array(_offsets())
    c = np.searchsorted(off, np.asarray(g), side="right") - 1
    return c.astype(np.int32), np.asarray(g) - off[c]


def _genome_rows(seed, n, splits):
    """rows over the three contigs in global coordinates (pads between
    contigs), strands + / -, with zero-width rows and rows that start or end
    exactly on a shard bound"""
    rng = np.random.default_rng(seed)
    off = _offsets()
    c = rng.integers(0, 3, n)
    L = np.array(_GENOME)[c]
    s = (rng.random(n) * (L - 600)).astype(np.int64)
    e = s + rng.integers(0, 600, n)
    gs, ge = np.array(off)[c] + s, np.array(off)[c] + e
    z = rng.random(n) < 0.05
    ge[z] = gs[z]
    # a zero-width row and a row ending exactly on every inner shard bound
    # (bounds off the pads), and a row starting there
    extra = []
    for b in splits[1:-1]:
        if b in off or b - 1 in [o - 1 for o in off[1:]]:
            continue
        extra += [(b, b), (b - 50, b), (b, b + 40)]
    if extra:
        gs = np.concatenate([gs, [x for x, _ in extra]])
        ge = np.concatenate([ge, [y for _, y in extra]])
    strand = rng.integers(1, 3, len(gs))
    return gs.astype(np.int64), ge.astype(np.int64), strand.astype(np.int64)


def _oracle_merge_global(gs, ge, strand=None):
    from oracle import oracle
    c, s = _to_local(gs)
    e = ge - np.array(_offsets())[c]
    return oracle.merge((c, s, e) if strand is None else (c, s, e, strand))


def _runs_global(m):
    off = np.array(_offsets())
    return off[m["contig"]] + m["start"], off[m["contig"]] + m["end"]


def _merge_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        from oracle import oracle
        span = _offsets()[-1]
        splits = ld.even_splits(span, world)
        n = 4000
        gs, ge, st = _genome_rows(9, n, splits)
        N = len(gs)
        sl = slice(rank * N // world, (rank + 1) * N // world)
        cols = [torch.from_numpy(x[sl].copy()) for x in (gs, ge, np.arange(N), st)]
        rgs, rge, rrow, rst = ld.route_rows(*cols[:3], splits, None, cols[3])
        lo, hi = splits[rank], splits[rank + 1]
        assert ((rgs >= lo) & (rgs < hi)).all()
        out = {}
        for stranded in (False, True):
            # the shard's local merge (the engine's, restated by the oracle),
            # rows in RegionOrdering, ties by row
            m = _oracle_merge_global(rgs.numpy(), rge.numpy(), rst.numpy() if stranded else None)
            a, b = _runs_global(m)
            runs = ld.TensorRuns(torch.from_numpy(a), torch.from_numpy(b),
                                 torch.from_numpy(m["strand"].astype(np.int64)) if stranded
                                 else None)
            table = ld.carry_table(runs, k=2, stranded=stranded)  # small k: the regather
            nr, drop, ext, _, _ = table[rank]
            kept = np.stack([a, b], 1)[drop:].copy()
            if ext is not None and len(kept):
                kept[-1, 1] = ext
            # every local row's global run (the Iterable[T] grouping)
            off = ld.run_offsets(table)[rank]
            gid = ld.global_run_ids(torch.from_numpy(m["run_of_row"]), drop, off)
            out[stranded] = (kept.tolist(), list(zip(rrow.tolist(), gid.tolist())))
            if not stranded:
                # this shard's share of the complement: its kept runs framed
                # by the previous shards' last end and the next first start
                prev_end, next_start = ld.complement_frame(table, rank)
                V = kept.tolist()
                if prev_end is not None:
                    V = [[prev_end, prev_end]] + V
                if next_start is not None:
                    V = V + [[next_start, next_start]]
                V = np.array(V, np.int64).reshape(-1, 2)
                c, s = _to_local(V[:, 0])
                e = V[:, 1] - np.array(_offsets())[c]
                comp = oracle.complement((c, s, e), _GENOME)
                gl = np.array(_offsets())[comp["contig"]] + comp["start"]
                gr = np.array(_offsets())[comp["contig"]] + comp["end"]
                mine = (gl >= lo) & (gl < hi)
                out["comp"] = list(zip(gl[mine].tolist(), gr[mine].tolist()))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_merge_run_ids_complement_strands(world):
    # the merge carry, global run ids of every row, the
    # complement's shard-bound gaps and the stranded carry, against the
    # unsharded oracle (shard-count invariant); zero-width rows and rows on
    # shard bounds included
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    span = _offsets()[-1]
    gs, ge, st = _genome_rows(9, 4000, ld.even_splits(span, world))
    for stranded in (False, True):
        m = _oracle_merge_global(gs, ge, st if stranded else None)
        a, b = _runs_global(m)
        runs = [tuple(x) for x in sum((r[1][stranded][0] for r in res), [])]
        assert runs == list(zip(a.tolist(), b.tolist()))
        ids = dict(sum((r[1][stranded][1] for r in res), []))
        assert [ids[i] for i in range(len(gs))] == m["run_of_row"].tolist()
    c, s = _to_local(gs)
    e = ge - np.array(_offsets())[c]
    comp = oracle.complement((c, s, e), _GENOME)
    off = np.array(_offsets())
    want = list(zip((off[comp["contig"]] + comp["start"]).tolist(),
                    (off[comp["contig"]] + comp["end"]).tolist()))
    got = sorted(sum((r[1]["comp"] for r in res), []))
    assert got == want


def _xsets_worker(rank, world, port, q, cap=None):
    if cap:  # rounds of at most `cap` bytes per rank pair (dist._a2a_payload)
        os.environ["LIME_A2A_MAX_BYTES"] = str(cap)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        # k sets, each rank holding rows for every destination (grouped by
        # destination, as lime_route_rows writes them); some (set, dest)
        # pairs empty
        k = 3
        sets, counts = [], []
        for i in range(k):
            c = [(rank + 2 * i + q) % 3 for q in range(world)]
            vals = [1000 * rank + 100 * i + 10 * q + j for q in range(world) for j in range(c[q])]
            t = torch.tensor(vals or [0], dtype=torch.int32)
            sets.append([t, -t])
            counts.append(c)
        got = ld.exchange_sets(sets, counts)
        out = [(cols[0][:m].tolist(), cols[1][:m].tolist(), m) for cols, m, _ in got]
        # the interleaved form (lime_route_rows_interleaved's [rows, 2]
        # buffers, received as per-rank slices): the same rows, same order
        gotr = ld.exchange_sets_rows([torch.stack(c, dim=1) for c in sets], counts)
        outr = []
        for slices, m, moved in gotr:
            t = torch.cat(slices) if slices else torch.empty((0, 2), dtype=torch.int32)
            outr.append((t[:, 0].tolist(), t[:, 1].tolist(), m))
        # one set through exchange_rows: the single-buffer exchange
        r1, rc = ld.exchange_rows(torch.stack(sets[1], dim=1), counts[1])
        one = (r1[:, 0].tolist(), r1[:, 1].tolist(), sum(rc))
        q.put((rank, out, outr, one))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cap", [(1, None), (2, None), (3, None), (2, 8), (3, 12)])
def test_exchange_sets(world, cap):
    # C5's batched exchange: every (source, set) segment lands in its set, in
    # rank order, both columns aligned; cap: payloads cut into rounds of a
    # few bytes per rank pair (the guard against RCCL's ~1 GiB message limit)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xsets_worker, args=(r, world, port, q, cap))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for me, got, gotr, one in res:
        for i, ((a, b, m), r) in enumerate(zip(got, gotr)):
            want = [1000 * p + 100 * i + 10 * me + j for p in range(world)
                    for j in range((p + 2 * i + me) % 3)]
            assert a == want and b == [-x for x in want] and m == len(want)
            assert r == (a, b, m)
        assert one == got[1]


# ---------------- count-balanced splitters (dist.splits_from_weighted_samples)
def _skewed(rank, world, n):
    """this rank's slice of two row sets over a 1e6-base span: set A puts 85 %
    of its rows in the first 5 % of the span (a pile-up region), set B is
    uniform; ranks hold unequal slices (rank r: (r + 1) parts)"""
    rng = np.random.default_rng(77)
    span = 1_000_000
    hot = rng.random(n) < 0.85
    a = np.where(hot, rng.integers(0, span // 20, n), rng.integers(0, span, n))
    b = rng.integers(0, span, n // 2)
    parts = sum(range(1, world + 1))
    lo = sum(range(1, rank + 1))

    def sl(x):
        m = len(x)
        return x[m * lo // parts:m * (lo + rank + 1) // parts]
    return span, sl(a), sl(b), a, b


def _balance_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        n, k = 60_000, 4096
        span, a, b, _, _ = _skewed(rank, world, n)
        rows = []
        for x in (a, b):  # evenly spaced samples of the unsorted rows, + the count
            t = torch.full((k + 1,), -1, dtype=torch.int64)
            if len(x):
                t[:k] = torch.from_numpy(x[(np.arange(k) * len(x)) // k].astype(np.int64))
            t[k] = len(x)
            rows.append(t)
        q.put((rank, ld.splits_from_weighted_samples(torch.stack(rows), span, world,
                                                     align=64)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sampled_splits_balance_rows(world):
    """coordinate-even shards put > 2x the mean rows on one shard here (1.5x
    at two shards, whose maximum is 2x); the sampled splitters every rank
    computes (the same on every rank) stay within 1.2x of the mean, over both
    sets together"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balance_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cuts = [r[1] for r in res]
    assert all(c == cuts[0] for c in cuts), "every rank derives the same splitters"
    splits = cuts[0]
    assert splits[0] == 0 and all(x % 64 == 0 for x in splits[1:-1])
    span, _, _, a, b = _skewed(0, world, 60_000)
    allg = np.concatenate([a, b])
    mean = len(allg) / world

    def counts(s):
        return np.histogram(allg, bins=s)[0]
    even = counts(ld.even_splits(span, world))
    assert even.max() > (1.5 if world == 2 else 2) * mean
    assert counts(splits).max() <= 1.2 * mean
