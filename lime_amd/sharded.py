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
