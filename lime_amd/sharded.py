"""Range-sharded operator step: one engine context per rank (one GPU per
process), rows exchanged with torch.distributed (RCCL over xGMI on MI355X,
gloo in CPU-side tests).  See lime_amd.dist for the protocol.

Coordinates: every rank's engine works in u32 global coordinates of its own
Space; `offset` places that space in a virtual int64 coordinate line shared
by all ranks (0 for one genome cut into ranges, r * span when every rank owns
its own copy of a genome -- the weak-scaling benchmark).  Boundary records
travel in virtual coordinates.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import dist as ld


class _EngineRuns:
    """merge result as seen by lime_amd.dist.merge_carry (virtual coordinates)."""

    def __init__(self, res, offset):
        self.res, self.off, self.n = res, offset, res.n
        self.last_end = -1
        if self.n:
            _, ge = res.copy_range(self.n - 1, 1)
            self.last_end = int(ge[0]) + offset

    def head(self, k):
        gs, ge = self.res.copy_range(0, k)
        return [int(x) + self.off for x in gs], [int(x) + self.off for x in ge]


class ShardStep:
    def __init__(self, ctx, space, offset=0, group=None, comm_device=None):
        self.ctx, self.space, self.offset, self.group = ctx, space, int(offset), group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.comm = comm_device if comm_device is not None else torch.device("cpu")
        self.dev = torch.device("cuda", ctx.device)

    # ------------------------------------------------------------- halo
    def _halo(self, sets, my_end):
        """right halo of every set: rows of later shards starting before this
        shard's max end.  Returns [(gs, ge, src_rank, src_row) int64 numpy]."""
        w, me = self.world, self.rank
        t = torch.tensor([my_end], dtype=torch.int64, device=self.comm)
        ends = torch.empty(w, dtype=torch.int64, device=self.comm)
        dist.all_gather_into_tensor(ends, t, group=self.group)
        ends = ends.tolist()
        out = []
        for S in sets:
            counts = []
            for r in range(w):
                key = ends[r] - self.offset
                if r < me and key > 0:
                    counts.append(S.lower_bound(min(key, 0xFFFFFFFF)))
                else:
                    counts.append(0)
            c = max(counts) if counts else 0
            if c:
                buf = torch.empty((3, c), dtype=torch.int32, device=self.dev)
                S.copy_rows_device(0, c, buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr())
                torch.cuda.synchronize(self.dev)
                u = buf.to(torch.int64) & 0xFFFFFFFF
                rows = torch.stack([u[0] + self.offset, u[1] + self.offset, u[2],
                                    torch.full_like(u[2], me)], dim=1)
                send = torch.cat([rows[:k] for k in counts]).to(self.comm)
            else:
                send = torch.empty((0, 4), dtype=torch.int64, device=self.comm)
            recv, _ = ld._alltoallv(send, counts, self.group)
            out.append(recv.cpu().numpy())
        return out

    def _extend(self, S, halo):
        """own sorted rows followed by the halo rows, as one engine set"""
        n, h = S.n, len(halo)
        gs = torch.empty(n + h, dtype=torch.int32, device=self.dev)
        ge = torch.empty(n + h, dtype=torch.int32, device=self.dev)
        row = torch.empty(n + h, dtype=torch.int32, device=self.dev)
        S.copy_rows_device(0, n, gs.data_ptr(), ge.data_ptr(), row.data_ptr())
        loc = halo[:, :2] - self.offset
        if loc.min() < 0 or loc.max() >= 2**32:
            raise ValueError("halo rows outside this shard's coordinate space")
        tail = np.stack([loc[:, 0], loc[:, 1], n + np.arange(h)]).astype(np.uint32)
        torch.cuda.synchronize(self.dev)
        t = torch.from_numpy(tail.view(np.int32)).to(self.dev)
        gs[n:], ge[n:], row[n:] = t[0], t[1], t[2]
        torch.cuda.synchronize(self.dev)
        E = self.ctx.set_from_global(self.space, n + h, gs.data_ptr(), ge.data_ptr(),
                                     row.data_ptr())
        return E

    # ------------------------------------------------------------- step
    def run(self, A, B, threshold=0, on_pairs=None):
        """A, B: this shard's own sorted sets.  Intersect (owned pairs only,
        emitted through on_pairs(plan, halo_rows)) + merge of A and B with the
        cross-shard carry.  Returns a dict of counts."""
        ctx = self.ctx
        ma, mb = ctx.merge(A), ctx.merge(B)
        ra, rb = _EngineRuns(ma, self.offset), _EngineRuns(mb, self.offset)
        my_end = max(ra.last_end, rb.last_end)
        halo_a, halo_b = self._halo([A, B], my_end)
        Ae = self._extend(A, halo_a) if len(halo_a) else A
        Be = self._extend(B, halo_b) if len(halo_b) else B
        plan = ctx.intersect(Ae, Be, threshold, a_owned=A.n, b_owned=B.n)
        if on_pairs is not None:
            on_pairs(plan, (halo_a, halo_b))
        da, ea = ld.merge_carry(ra, group=self.group, device=self.comm)
        db, eb = ld.merge_carry(rb, group=self.group, device=self.comm)
        out = {"pairs": plan.n, "runs_a": ma.n - da, "runs_b": mb.n - db,
               "drop": (da, db), "extend": (ea, eb), "halo": (len(halo_a), len(halo_b)),
               "merge_a": ma, "merge_b": mb}
        plan.close()
        for E, S in ((Ae, A), (Be, B)):
            if E is not S:
                E.close()
        return out


class ShardedAnd:
    """BASELINE C5: k-way intersection over bit-per-base sets, range-sharded.

    Shard r (one rank per GPU) owns global coordinates [splits[r],
    splits[r+1]) (lime_amd.dist.coord_splits).  Per input set every rank
    routes its slice of unsorted rows to the shards they overlap, clipped at
    the shard bounds (lime_route_rows, clip = 1: exact for base-level
    algebra, no halo); one all_to_all moves them (RCCL over
    xGMI, device buffers); each shard paints the rows it received into a
    bitset over its window (lime_bitset_from_global) and ANDs the k bitsets
    (lime_bitset_and_runs).  Runs are in global coordinates; the one
    boundary fix-up (a run ending exactly at a shard bound continues in the
    next shard) is dist.bitset_carry, one all_gather of 4 numbers per shard.
    The runs stay sharded; run(gather=True) adds the emulated allgatherv.
    Same code at world size 1 (no collective is issued then).

    Reference analogue: the range partitioning + replication of
    OverlapBasedSetTheory.scala:74-84 (here each right record is clipped, not
    replicated) and SURVEY.md Appendix A.4 (N-way = fold of intersect over
    merged operands, per base).
    """

    def __init__(self, ctx, space, splits=None, group=None, comm_device=None,
                 shared_stream=False):
        self.ctx, self.space, self.group = ctx, space, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.splits = splits or ld.coord_splits(space.span, self.world)
        self.lo, self.hi = self.splits[self.rank], self.splits[self.rank + 1]
        self.dev = torch.device("cuda", ctx.device)
        self.comm = comm_device
        # the engine shares torch's current stream (bench): stream order
        # covers the collectives; otherwise drain around them
        self.shared = shared_stream
        self.moved = 0  # rows received from other shards (diagnostics)

    def _sync(self):
        if not self.shared:
            self.ctx.synchronize()
            torch.cuda.current_stream(self.dev).synchronize()

    def bitset(self, n, d_contig, d_start, d_end):
        """this shard's bitset of one set, from this rank's slice of its rows"""
        ctx, sp = self.ctx, self.space
        if self.world == 1:
            return ctx.bitset_from_device(sp, n, d_contig, d_start, d_end)
        cap = n + 4096
        gs = torch.empty(cap, dtype=torch.int32, device=self.dev)
        ge = torch.empty(cap, dtype=torch.int32, device=self.dev)
        counts = ctx.route_rows(sp, n, d_contig, d_start, d_end, self.splits, clip=True,
                                cap=cap, d_gs=gs.data_ptr(), d_ge=ge.data_ptr())
        if sum(counts) > cap:  # many rows cross shard bounds: exact size
            cap = sum(counts)
            gs = torch.empty(cap, dtype=torch.int32, device=self.dev)
            ge = torch.empty(cap, dtype=torch.int32, device=self.dev)
            counts = ctx.route_rows(sp, n, d_contig, d_start, d_end, self.splits, clip=True,
                                    cap=cap, d_gs=gs.data_ptr(), d_ge=ge.data_ptr())
        self._sync()
        (rgs, rge), rc = ld.exchange([gs, ge], counts, self.group, self.comm)
        self._sync()
        self.moved += sum(rc) - rc[self.rank]
        m = sum(rc)
        return ctx.bitset_from_global(sp, self.lo, self.hi, m, rgs.data_ptr(), rge.data_ptr())

    def run(self, inputs, gather=False):
        """inputs: [(n, d_contig, d_start, d_end)] per set (this rank's rows,
        device pointers).  Returns a dict: the shard's AND result (global
        coordinates), the carry (drop_first, new_last_end), the total run
        count of the unsharded result and, with gather=True, every run as an
        int64 [m, 2] tensor (global start, end) in order."""
        bits = [self.bitset(*x) for x in inputs]
        res = self.ctx.bitset_and(bits)
        for b in bits:
            b.close()
        n = res.n
        drop, ext = 0, None
        total = n
        if self.world > 1:
            fs = fe = le = -1
            if n:
                gs0, ge0 = res.copy_range(0, 1)
                fs, fe = int(gs0[0]), int(ge0[0])
                _, gel = res.copy_range(n - 1, 1)
                le = int(gel[0])
            drop, ext = ld.bitset_carry(n, fs, fe, le, self.group, self.comm or self.dev)
            cd = self.comm or self.dev
            t = torch.tensor([n - drop], dtype=torch.int64, device=cd)
            dist.all_reduce(t, group=self.group)
            total = int(t.item())
        out = {"result": res, "drop": drop, "extend": ext, "runs_total": total,
               "window": (self.lo, self.hi)}
        if gather:
            gs, ge = res.copy_range(0, n) if n else (np.zeros(0, np.uint32),) * 2
            runs = np.stack([gs.astype(np.int64), ge.astype(np.int64)], axis=1)[drop:]
            if ext is not None and len(runs):
                runs[-1, 1] = ext
            t = torch.from_numpy(np.ascontiguousarray(runs))
            if self.world > 1:
                t, _ = ld.allgatherv(t.to(self.comm or self.dev), self.group, self.comm)
            out["runs"] = t.cpu()
        return out
