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
