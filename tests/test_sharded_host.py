"""Host logic of lime_amd.sharded.ShardStep on the CPU: gloo, world 2 and 3,
with a numpy/oracle stand-in for the engine context (this container has no
GPU).  The GPU version of the same check is tests/test_gpu_sharded.py."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

LENS = [300_000, 200_000, 250_000]
NAMES = ["c0", "c1", "c2"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeSpace:
    def __init__(self):
        self.names, self.lengths = NAMES, np.array(LENS)
        self.offsets = np.concatenate([[0], np.cumsum(np.array(LENS) + 1)])
        self.span = int(self.offsets[-1])


class FakeSet:
    """sorted rows in global coordinates with row ids (the engine's lime_set)"""

    def __init__(self, gs, ge, row):
        o = np.lexsort((row, ge > gs, gs))
        self.gs, self.ge, self.row = gs[o], ge[o], row[o]
        self.n = len(gs)

    def lower_bound(self, key):
        return int(np.searchsorted(self.gs, key, "left"))

    def lower_bounds(self, keys):
        return [self.lower_bound(k) for k in keys]

    def stats(self):
        w = self.ge - self.gs
        return (int(w.min()) if self.n else 0, int(w.max()) if self.n else 0,
                bool((w == 0).any()))

    def copy_rows_device(self, first, count, d_gs, d_ge, d_row):
        for src, dst in ((self.gs, d_gs), (self.ge, d_ge), (self.row, d_row)):
            a = np.ascontiguousarray(src[first:first + count], dtype=np.uint32)
            ctypes.memmove(dst, a.ctypes.data, 4 * count)

    def close(self):
        pass


class FakeRuns:
    def __init__(self, gs, ge):
        self.gs, self.ge, self.n = gs, ge, len(gs)

    def copy_range(self, first, count):
        return (self.gs[first:first + count].astype(np.uint32),
                self.ge[first:first + count].astype(np.uint32))

    def copy_rows_device(self, first, count, d_gs, d_ge):
        for src, dst in ((self.gs, d_gs), (self.ge, d_ge)):
            a = np.ascontiguousarray(src[first:first + count], dtype=np.uint32)
            ctypes.memmove(dst, a.ctypes.data, 4 * count)

    def close(self):
        pass


class FakePlan:
    def __init__(self, pairs):
        self.pairs, self.n = pairs, len(pairs)

    def close(self):
        pass


class FakeCtx:
    device = 0

    def synchronize(self):
        pass

    def merge(self, S):
        from oracle import oracle
        m = oracle.merge((np.zeros(S.n, np.int32), S.gs, S.ge))
        return FakeRuns(m["start"], m["end"])

    def set_from_global(self, space, n, d_gs, d_ge, d_row):
        def arr(p):
            return np.ctypeslib.as_array((ctypes.c_uint32 * n).from_address(p)).astype(np.int64)
        return FakeSet(arr(d_gs), arr(d_ge), arr(d_row))

    def set_extend_sorted(self, S, n, d_gs, d_ge, d_row, min_w, max_w, zero):
        def arr(p):
            return np.ctypeslib.as_array((ctypes.c_uint32 * n).from_address(p)).astype(np.int64)
        g, e, r = arr(d_gs), arr(d_ge), arr(d_row)
        # (own rows start below the shard's upper split, halo rows at or past it)
        assert n == 0 or S.n == 0 or g[0] > S.gs[-1], "halo rows start past the shard's rows"
        w = e - g
        assert n == 0 or (w.max() <= max_w and w.min() >= min_w and (zero or not (w == 0).any()))
        return FakeSet(np.concatenate([S.gs, g]), np.concatenate([S.ge, e]),
                       np.concatenate([S.row, r]))

    def intersect(self, A, B, t, a_owned, b_owned):
        from oracle import oracle
        r = oracle.intersect((np.zeros(A.n, np.int32), A.gs, A.ge),
                             (np.zeros(B.n, np.int32), B.gs, B.ge), t)
        ai, bi = r["a_row"], r["b_row"]  # sorted-position indices
        a_owns = A.gs[ai] <= B.gs[bi]
        keep = np.where(a_owns, ai < a_owned, bi < b_owned)
        return FakePlan(list(zip(A.row[ai[keep]].tolist(), B.row[bi[keep]].tolist())))


def _rows():
    from lime_amd import synth
    A = synth.uniform(LENS, 4000, 0x11, 10, 6000)
    B = synth.uniform(LENS, 3000, 0x22, 10, 9000)
    return A, B


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        from lime_amd import dist as ld
        from lime_amd import sharded
        torch.cuda.synchronize = lambda *a, **k: None  # CPU stand-in
        sp = FakeSpace()
        off = sp.offsets
        A, B = _rows()
        splits = ld.even_splits(sp.span, world)

        def owned(X):
            g = off[X[0]] + X[1]
            return [np.nonzero((g >= splits[r]) & (g < splits[r + 1]))[0] for r in range(world)]
        own_a, own_b = owned(A), owned(B)
        ia, ib = own_a[rank], own_b[rank]

        def mk(X, idx):  # the shard's own rows, global row ids (as load() delivers them)
            c = X[0][idx]
            return FakeSet(off[c] + X[1][idx], off[c] + X[2][idx], idx.astype(np.int64))
        Aset, Bset = mk(A, ia), mk(B, ib)
        step = sharded.ShardStep(FakeCtx(), sp, splits=splits, comm_device=torch.device("cpu"),
                                 shared_stream=True)
        step.dev = torch.device("cpu")
        got = []

        def on_pairs(plan):  # halo rows carry their global ids: pairs name input rows
            got.extend((int(a), int(b)) for a, b in plan.pairs)
        out = step.run(Aset, Bset, on_pairs=on_pairs)
        runs = []
        for k, res in enumerate((out["merge_a"], out["merge_b"])):
            d, e = out["drop"][k], out["extend"][k]
            gs, ge = list(res.gs[d:]), list(res.ge[d:])
            if e is not None and gs:
                ge[-1] = e
            runs.append(list(zip(gs, ge)))
        q.put((rank, got, runs, out["halo"]))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc(), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_step_host_logic(world):
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[1] == "error"]
    assert not errs, errs[0]
    A, B = _rows()
    exp = oracle.intersect(A, B)
    assert sorted(sum((r[1] for r in res), [])) == \
        sorted(zip(exp["a_row"].tolist(), exp["b_row"].tolist()))
    assert sum(r[3][0] + r[3][1] for r in res) > 0
    off = FakeSpace().offsets
    for k, X in ((0, A), (1, B)):
        m = oracle.merge(X)
        runs = sum((r[2][k] for r in res), [])
        want = [(int(off[c] + s), int(off[c] + e)) for c, s, e in
                zip(m["contig"], m["start"], m["end"])]
        assert [(int(a), int(b)) for a, b in runs] == want
