"""Range-sharded operator steps: one engine context per rank (one GPU per
process), rows exchanged with torch.distributed (RCCL over xGMI on MI355X;
gloo, staged through the host, in CPU-side tests and one-GPU rehearsals).
See lime_amd.dist for the protocol.

One genome is cut into coordinate ranges (dist.even_splits / coord_splits /
sample_splits); shard r owns the rows whose global start lies in
[splits[r], splits[r+1]).  Row ids are global (the caller's row_base + input
index), so every output record names its input rows directly.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import dist as ld


SAMPLES = 4096  # start samples per rank and input set for sampled splitters


def _sampled_splits(step, inputs, align):
    """dist.splits_from_weighted_samples over the engine's samples of the
    inputs [(n, d_contig, d_start, ...)] of this rank"""
    k = SAMPLES
    rows = []
    for x in inputs:
        n, d_contig, d_start = int(x[0]), x[1], x[2]
        t = torch.full((k + 1,), -1, dtype=torch.int64, device=step.dev)
        if n:
            buf = torch.empty(k, dtype=torch.int32, device=step.dev)
            step.ctx.sample_starts(step.space, n, d_contig, d_start, k, buf.data_ptr())
            step._sync()  # engine output -> torch
            t[:k] = buf.to(torch.int64) & 0xFFFFFFFF
        t[k] = n
        rows.append(t)
    cd = step.comm if step.comm is not None else step.dev
    s = torch.stack(rows).to(cd)
    return ld.splits_from_weighted_samples(s, step.space.span, step.world, step.group, align)


class _EngineRuns:
    """merge result as seen by lime_amd.dist.carry_tables: its leading runs
    and last end copied on the device into the gathered words (payload), so
    the carry costs no host copy before its one all_gather"""

    def __init__(self, res, stranded=False, sync=None, dev=None):
        self.res, self.n, self.stranded = res, res.n, stranded
        self._sync = sync or (lambda: None)
        self.dev = dev  # the engine's device (where the copies land)
        self.last_strand = 0
        if self.n and stranded:
            self.last_strand = int(res.run_strands(self.n - 1, 1)[0])

    @property
    def last_end(self):
        if not self.n:
            return -1
        _, ge = self.res.copy_range(self.n - 1, 1)
        return int(ge[0])

    def head(self, k):
        gs, ge = self.res.copy_range(0, k)
        return [int(x) for x in gs], [int(x) for x in ge]

    def head_strands(self, k):
        return [int(x) for x in self.res.run_strands(0, k)]

    def payload(self, k, dev):
        """n, last end, last strand, the first k runs' starts, ends, strands
        (int64 on `dev`; -1 past the runs)"""
        n, kk = self.n, min(k, self.n)
        out = torch.full((3 * k + 3,), -1, dtype=torch.int64, device=dev)
        out[0] = n
        out[2] = self.last_strand if self.stranded and n else 0
        if n:
            g = torch.empty(kk + 1, dtype=torch.int32, device=self.dev)
            e = torch.empty(kk + 1, dtype=torch.int32, device=self.dev)
            self.res.copy_rows_device(0, kk, g.data_ptr(), e.data_ptr())
            self.res.copy_rows_device(n - 1, 1, g[kk:].data_ptr(), e[kk:].data_ptr())
            self._sync()  # the engine's copies land before torch reads them
            g64 = (g.to(torch.int64) & 0xFFFFFFFF).to(dev)
            e64 = (e.to(torch.int64) & 0xFFFFFFFF).to(dev)
            out[1] = e64[kk]
            out[3:3 + kk] = g64[:kk]
            out[3 + k:3 + k + kk] = e64[:kk]
            if self.stranded:
                out[3 + 2 * k:3 + 2 * k + kk] = torch.tensor(self.head_strands(kk),
                                                             dtype=torch.int64, device=dev)
        return out


class ShardStep:
    """Pairwise intersect + merge of both inputs over one range shard.

    load():  this rank's slice of unsorted rows -> the rows this shard owns,
             sorted (lime_route_rows, clip = 0: a row goes to the shard of its
             start; one all_to_all per array -- the Spark shuffle of ADAM
             repartitionAndSort, cli/Intersection.scala:42-43)
    run():   merge both sets locally; right halo (rows of later shards that
             start before this shard's max end: the replication of
             OverlapBasedSetTheory.scala:75-80, bounded by the longest row) by
             one all_gather of ends + one all_to_all of device rows; intersect
             with ownership (a pair belongs to the row with the smaller start,
             ties to a, so shard outputs are disjoint); merge carry (one
             all_gather replaces SetTheory.scala:236-282's log2(P) rounds).
    """

    def __init__(self, ctx, space, splits=None, group=None, comm_device=None,
                 shared_stream=False):
        """splits: the shard bounds; None = count-balanced, sampled from the
        inputs (plan_splits, or the first load's rows) -- equal coordinate
        ranges are not equal work on real BED density or C3's pile-ups"""
        self.ctx, self.space, self.group = ctx, space, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.splits = splits
        self.comm = comm_device
        self.dev = torch.device("cuda", ctx.device)
        self.shared = shared_stream
        self.routed = 0  # rows received from other ranks by load() (diagnostics)

    def _sync(self):
        if not self.shared:
            self.ctx.synchronize()
            torch.cuda.current_stream(self.dev).synchronize()

    def _i32(self, n):
        return torch.empty(max(int(n), 1), dtype=torch.int32, device=self.dev)

    def _need_splits(self, what):
        if self.splits is None:
            raise RuntimeError(f"ShardStep.{what}: no shard bounds yet -- call "
                               "plan_splits(inputs) with every input set first (or load())")

    # ----------------------------------------------------------- routing
    def plan_splits(self, inputs):
        """count-balanced shard bounds from this rank's inputs [(n, d_contig,
        d_start, ...)] (unsorted device rows; d_contig None: global starts):
        SAMPLES evenly spaced starts per set (lime_sample_starts), one
        all_gather, the weighted quantiles (dist.splits_from_weighted_samples)"""
        self.splits = _sampled_splits(self, inputs, 1)
        return self.splits

    def route(self, n, d_contig, d_start, d_end, row_base=0, d_strand=None):
        """this rank's slice of unsorted rows -> the rows this shard owns:
        [gs, ge, row(, strand)] int32 device tensors (global coordinates and
        row ids), one packed all_to_all (lime_route_rows + dist.exchange).
        Without planned bounds only the first routed set is sampled: callers
        with several inputs (run(A, B), subtract) should call plan_splits with
        all of them first, as bench.py does, so that skew in any is balanced."""
        ctx, sp = self.ctx, self.space
        if self.splits is None:
            self.plan_splits([(n, d_contig, d_start)])
        if not d_strand:
            # interleaved: the route writes the all_to_all send buffer itself
            # and one device pass splits the received rows into columns (the
            # column form stacked them before the collective, 24 B per routed
            # row, and copied each column out after it, ~48 B)
            buf = torch.empty((max(int(n), 1), 3), dtype=torch.int32, device=self.dev)
            counts = ctx.route_rows_interleaved(sp, n, d_contig, d_start, d_end, self.splits, 3,
                                                buf.data_ptr(), clip=False, cap=n,
                                                row_base=row_base)
            self._sync()  # engine output -> the collective
            recv, rc = ld.exchange_rows(buf, counts, self.group, self.comm)
            del buf
            m = recv.shape[0]
            cols = [self._i32(m) for _ in range(3)]
            self._sync()  # the collective's output -> the engine
            if m:
                ctx.deinterleave(m, 3, recv.data_ptr(), *(c.data_ptr() for c in cols))
            self._sync()
            del recv
            self.routed += sum(rc) - rc[self.rank]
            return [c[:m] for c in cols]
        cols = [self._i32(n) for _ in range(4 if d_strand else 3)]
        st8 = torch.empty(max(int(n), 1), dtype=torch.int8, device=self.dev) if d_strand else None
        counts = ctx.route_rows(sp, n, d_contig, d_start, d_end, self.splits, clip=False, cap=n,
                                d_gs=cols[0].data_ptr(), d_ge=cols[1].data_ptr(),
                                d_row=cols[2].data_ptr(), row_base=row_base, d_strand=d_strand,
                                d_strand_out=st8.data_ptr() if d_strand else None)
        self._sync()  # engine output -> torch ops
        if d_strand:
            cols[3] = st8.to(torch.int32)
        recv, rc = ld.exchange(cols, counts, self.group, self.comm, packed=True)
        self._sync()
        self.routed += sum(rc) - rc[self.rank]
        return recv

    def load(self, n, d_contig, d_start, d_end, row_base=0, d_strand=None):
        """-> IntervalSet of the rows this shard owns (global row ids); with
        strand codes (int8 per input row) a stranded set: full RegionOrdering,
        merge breaks runs at strand changes (cli/Intersection.scala:45,48
        key both sides with ReferenceRegion.stranded, Merge.scala:19)"""
        recv = self.route(n, d_contig, d_start, d_end, row_base, d_strand)
        m = recv[0].numel()
        if d_strand:
            st8 = recv[3].to(torch.int8)
            self._sync()  # torch output -> engine input
            S = self.ctx.set_from_global_stranded(self.space, m, recv[0].data_ptr(),
                                                  recv[1].data_ptr(), recv[2].data_ptr(),
                                                  st8.data_ptr())
        else:
            S = self.ctx.set_from_global(self.space, m, *(t.data_ptr() for t in recv[:3]))
        return S

    def load_strand_groups(self, n, d_contig, d_start, d_end, d_strand, row_base=0):
        """stranded rows -> {strand code: IntervalSet} of this shard's rows:
        the pairwise ops pair equal strands only (ReferenceRegion.overlaps),
        so each strand group runs through the strand-free kernels"""
        gs, ge, row, st = self.route(n, d_contig, d_start, d_end, row_base, d_strand)
        out = {}
        codes = torch.unique(st).tolist() if st.numel() else []
        for c in codes:
            keep = st == c
            sub = [x[keep].contiguous() for x in (gs, ge, row)]
            self._sync()
            out[int(c)] = self.ctx.set_from_global(self.space, sub[0].numel(),
                                                   *(t.data_ptr() for t in sub))
        return out

    # -------------------------------------------------------------- halo
    def _halo(self, sets, ends=None, my_end=-1):
        """right halo of every set, on the device: [(gs, ge, row) int32
        tensors], each sorted (later shards' prefixes in rank order).  `ends`:
        every shard's max row end, when the caller gathered them already;
        else one all_gather of `my_end`.  Every set's rows travel in ONE
        packed all_to_all (dist.exchange_sets)."""
        w, me = self.world, self.rank
        cd = self.comm if self.comm is not None else self.dev
        if ends is None:
            t = torch.empty(w, dtype=torch.int64, device=cd)
            dist.all_gather_into_tensor(t, torch.tensor([my_end], dtype=torch.int64, device=cd),
                                        group=self.group)
            ends = t.tolist()
        cols, counts = [], []
        for S in sets:
            # rows of mine that shard r < me needs: gs < ends[r] (one batched
            # search for every earlier shard)
            ask = [r for r in range(w) if r < me and ends[r] > 0]
            got = dict(zip(ask, S.lower_bounds([min(ends[r], 0xFFFFFFFF) for r in ask])))
            cnt = [got.get(r, 0) for r in range(w)]
            c = max(cnt) if cnt else 0
            pre = [self._i32(c) for _ in range(3)]
            if c:
                S.copy_rows_device(0, c, *(t.data_ptr() for t in pre))
            cols.append(pre)
            counts.append(cnt)
        self._sync()  # the engine's copies land before torch.cat reads them
        send = [[torch.cat([t[:k] for k in cnt]) if sum(cnt) else t[:0] for t in pre]
                for pre, cnt in zip(cols, counts)]
        got = ld.exchange_sets(send, counts, self.group, self.comm)
        self._sync()
        return [recv for recv, _, _ in got]

    def _extend(self, S, halo, widths):
        """own sorted rows followed by the halo rows (already in order: later
        shards' rows start past every own row) as one engine set, copied on
        the device without a sort, a validation or a read-back
        (lime_set_extend_sorted); `widths` bounds the halo rows' widths (min,
        max, any zero-width) -- the sending shards' set statistics"""
        h = halo[0].numel()
        return self.ctx.set_extend_sorted(S, h, *(t.data_ptr() for t in halo[:3]), *widths)

    def _left_halo(self, S):
        """rows of earlier shards that may reach into this shard: shard q
        sends shard r > q its sorted rows from the first one whose running max
        end passes split[r] (a superset of the rows overlapping r's range;
        extra rows overlap nothing there).  Device rows, in order."""
        w, me = self.world, self.rank
        self._need_splits("subtract")
        later = list(range(me + 1, w))
        got = dict(zip(later, S.first_reachings([min(self.splits[r], 0xFFFFFFFF)
                                                 for r in later])))
        first = [got.get(r, S.n) for r in range(w)]
        counts = [S.n - f for f in first]
        f0 = min(first) if first else S.n
        c = S.n - f0
        suf = [self._i32(c) for _ in range(3)]
        if c:
            S.copy_rows_device(f0, c, *(t.data_ptr() for t in suf))
            self._sync()
        send = [torch.cat([t[first[r] - f0:] for r in range(w) if counts[r]])
                if sum(counts) else t[:0] for t in suf]
        self._sync()
        recv, _ = ld.exchange(send, counts, self.group, self.comm)
        self._sync()
        return recv

    def subtract(self, A, B, threshold=0, mode=0):
        """DistributedSubtract of this shard's own rows of A: every B row that
        overlaps one of them -- the left halo (earlier shards' rows reaching
        in) + own B rows + the right halo -- as one sorted set, joined on the
        device without a sort or a read-back (lime_set_concat_sorted).
        Outputs are disjoint across shards (each A row is subtracted where it
        is owned) and carry global row ids (Subtract.scala:78-116 over the
        replication of OverlapBasedSetTheory.scala:75-80).  The right halo
        reaches to A's last start + A's widest row (no merge of A), and every
        shard's bound and B width statistics travel in ONE all_gather."""
        w, me = self.world, self.rank
        cd = self.comm if self.comm is not None else self.dev
        amin, amax, _ = A.stats()
        bmin, bmax, bz = B.stats()
        # [A's reach (the right halo bound), B's min width, max width, zero]
        mine = torch.tensor([-1, bmin, bmax, int(bz)] if B.n else [-1, 1 << 32, 0, 0],
                            dtype=torch.int64, device=self.dev)
        if A.n:
            # (the unused end / row destinations stay referenced until the
            # sync: the engine's copy lands in them asynchronously)
            g, ge_scratch, row_scratch = self._i32(1), self._i32(1), self._i32(1)
            A.copy_rows_device(A.n - 1, 1, g.data_ptr(), ge_scratch.data_ptr(),
                               row_scratch.data_ptr())
            self._sync()
            del ge_scratch, row_scratch
            mine[0] = (g[0].to(torch.int64) & 0xFFFFFFFF) + amax
        t = torch.empty(w * 4, dtype=torch.int64, device=cd)
        dist.all_gather_into_tensor(t, mine.to(cd), group=self.group)
        tab = t.view(w, 4).tolist()
        left = self._left_halo(B)
        (right,) = self._halo([B], ends=[x[0] for x in tab])
        n, hl, hr = B.n, left[0].numel(), right[0].numel()
        if hl or hr:
            # the halo rows' widths are bounded by their shards' statistics
            src = [x for q, x in enumerate(tab) if q != me and x[2] >= x[1]]
            wmin = min([x[1] for x in src], default=0)
            wmax = max([x[2] for x in src], default=0)
            zero = any(x[3] for x in src)
            self._sync()
            Be = self.ctx.set_concat_sorted((hl, *(c.data_ptr() for c in left)), B,
                                            (hr, *(c.data_ptr() for c in right)),
                                            min(wmin, 0xFFFFFFFF), wmax, zero)
        else:
            Be = B
        res = self.ctx.subtract(A, Be, threshold, mode)
        return res, (hl, hr), Be

    # ------------------------------------------------ merge / complement
    def merge(self, S, stranded=False):
        """DistributedMerge over the shards (SetTheory.scala:202-282): the
        local merge, then ONE all_gather (dist.carry_table).  Returns a dict:
        the local result, drop / ext (this shard drops its first `drop` runs
        and ends its last at `ext`), `offset` (the global index of its first
        kept run) and the table of every shard."""
        res = self.ctx.merge(S)
        cd = self.comm if self.comm is not None else self.dev
        table = ld.carry_table(_EngineRuns(res, stranded, self._sync, self.dev), self.group,
                               device=cd, stranded=stranded)
        nr, drop, ext, _, _ = table[self.rank]
        return {"result": res, "drop": drop, "ext": ext, "table": table,
                "offset": ld.run_offsets(table)[self.rank], "runs": nr - drop}

    def global_run_ids(self, m, n_rows):
        """(row ids, global run ids) of this shard's rows, int64 device
        tensors: the Iterable[T] grouping of the sharded merge (SetTheory.scala
        :213-217 after the moves of :263-272)"""
        run, row = self._i32(n_rows), self._i32(n_rows)
        if n_rows:
            m["result"].copy_run_ids_device(run.data_ptr(), row.data_ptr())
            self._sync()
        local = run[:n_rows].to(torch.int64) & 0xFFFFFFFF
        return (row[:n_rows].to(torch.int64) & 0xFFFFFFFF,
                ld.global_run_ids(local, m["drop"], m["offset"]))

    def complement(self, S, m=None):
        """This shard's share of DistributedComplement (Complement.scala
        :33-134) against the shard space's contigs: the gaps that START in its
        window [split[r], split[r+1]), from its carried runs framed by the
        previous shards' last run end and the next shards' first run start
        (the gap at a partition bound, :67-73 / :112-122; contigs without
        data, :39-45, fall to the shard holding their start).  The shards'
        gaps concatenate to the unsharded result.  `m`: this shard's merge()
        of S when the caller has it (kept open), else merged here."""
        self._need_splits("complement")
        own = m is None
        if own:
            m = self.merge(S)
        res, drop, ext = m["result"], m["drop"], m["ext"]
        prev_end, next_start = ld.complement_frame(m["table"], self.rank)
        k = res.n - drop
        lead = 1 if prev_end is not None else 0
        tot = lead + k + (1 if next_start is not None else 0)
        gs, ge = self._i32(tot), self._i32(tot)
        if k:
            res.copy_rows_device(drop, k, gs[lead:].data_ptr(), ge[lead:].data_ptr())
            self._sync()  # before torch overwrites the last end
        if prev_end is not None:
            gs[0] = ge[0] = prev_end - (1 << 32) if prev_end >= (1 << 31) else prev_end
        if ext is not None and k:
            ge[lead + k - 1] = ext - (1 << 32) if ext >= (1 << 31) else ext
        if next_start is not None:
            v = next_start - (1 << 32) if next_start >= (1 << 31) else next_start
            gs[tot - 1] = ge[tot - 1] = v
        self._sync()
        out = self.ctx.complement_runs(self.space, tot, gs.data_ptr(), ge.data_ptr(),
                                       self.splits[self.rank], self.splits[self.rank + 1])
        if own:
            res.close()
        return out

    # -------------------------------------------------------------- step
    def run(self, A, B, threshold=0, on_pairs=None):
        """A, B: this shard's own sorted sets (load()).  Intersect (owned
        pairs only, handed to on_pairs(plan)) + merge of A and B with the
        cross-shard carry.  Returns a dict of counts and the merge results."""
        ctx = self.ctx
        ma, mb = ctx.merge(A), ctx.merge(B)
        ra = _EngineRuns(ma, sync=self._sync, dev=self.dev)
        rb = _EngineRuns(mb, sync=self._sync, dev=self.dev)
        cd = self.comm if self.comm is not None else self.dev
        # ONE all_gather: both sets' merge carries, every shard's last run
        # ends (its rows' max end: the halo bound) and width bounds
        wa, wb = A.stats(), B.stats()
        (ta, tb), ex, (la, lb) = ld.carry_tables(
            [ra, rb], self.group, device=cd,
            extra=[wa[0], wa[1], int(wa[2]), wb[0], wb[1], int(wb[2])])
        ends = [max(x, y) for x, y in zip(la, lb)]
        later = ex[self.rank + 1:]  # the halo rows come from later shards
        wha = (min([x[0] for x in later], default=0), max([x[1] for x in later], default=0),
               any(x[2] for x in later))
        whb = (min([x[3] for x in later], default=0), max([x[4] for x in later], default=0),
               any(x[5] for x in later))
        halo_a, halo_b = self._halo([A, B], ends=ends)
        Ae = self._extend(A, halo_a, wha) if halo_a[0].numel() else A
        Be = self._extend(B, halo_b, whb) if halo_b[0].numel() else B
        plan = ctx.intersect(Ae, Be, threshold, a_owned=A.n, b_owned=B.n)
        if on_pairs is not None:
            on_pairs(plan)
        da, ea = ta[self.rank][1], ta[self.rank][2]
        db, eb = tb[self.rank][1], tb[self.rank][2]
        out = {"pairs": plan.n, "runs_a": ma.n - da, "runs_b": mb.n - db,
               "drop": (da, db), "extend": (ea, eb),
               "halo": (halo_a[0].numel(), halo_b[0].numel()), "merge_a": ma, "merge_b": mb}
        plan.close()
        for E, S in ((Ae, A), (Be, B)):
            if E is not S:
                E.close()
        return out


class ShardedBitset:
    """Bit-per-base set algebra range-sharded (BASELINE C4 and C5): k-way
    intersection (C5), complement and difference (C4).

    Shard r (one rank per GPU) owns global coordinates [splits[r],
    splits[r+1]) (lime_amd.dist.coord_splits).  Per input set every rank
    routes its slice of unsorted rows to the shards they overlap, clipped at
    the shard bounds (lime_route_rows, clip = 1: exact for base-level
    algebra, no halo); one all_to_all moves them (RCCL over
    xGMI, device buffers); each shard bins the rows it received and paints
    and ANDs all k sets tile by tile in one kernel over its window
    (lime_bitset_and_from_global; NOT / AND-NOT paint per-set bitsets,
    lime_bitset_from_global).  Runs are in global coordinates; the one
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
        self.dev = torch.device("cuda", ctx.device)
        self.comm = comm_device
        # splits None: count-balanced, sampled from the first run's inputs and
        # aligned to the bitset bin (at world 1 the whole genome)
        self.splits = splits if splits or self.world > 1 else ld.coord_splits(space.span, 1)
        self.lo, self.hi = (self.splits[self.rank], self.splits[self.rank + 1]) if self.splits \
            else (None, None)
        # the engine shares torch's current stream (bench): stream order
        # covers the collectives; otherwise drain around them
        self.shared = shared_stream
        self.moved = 0  # rows received from other shards (diagnostics)

    def _sync(self):
        if not self.shared:
            self.ctx.synchronize()
            torch.cuda.current_stream(self.dev).synchronize()

    def plan_splits(self, inputs):
        """count-balanced shard windows from this rank's inputs [(n, d_contig,
        d_start, d_end)] (ShardStep.plan_splits), bounds aligned to the bitset
        bin (dist.bitset_align)"""
        self.splits = _sampled_splits(self, inputs, ld.bitset_align(self.space.span, self.world))
        self.lo, self.hi = self.splits[self.rank], self.splits[self.rank + 1]
        return self.splits

    def _i32(self, n):
        return torch.empty(max(int(n), 1), dtype=torch.int32, device=self.dev)

    def _ensure_splits(self, inputs):
        """the shard windows, sampled from `inputs` when none were given
        (collective: every rank calls the same entry point)"""
        if self.splits is None:
            self.plan_splits(inputs)

    def shard_rows(self, n, d_contig, d_start, d_end):
        """this rank's slice of one set's rows -> the rows of this shard's
        window from every rank (global coordinates, clipped): (m, gs, ge)"""
        self._ensure_splits([(n, d_contig, d_start, d_end)])
        buf, counts = self._route_clipped(n, d_contig, d_start, d_end)
        self._sync()
        recv, rc = ld.exchange_rows(buf, counts, self.group, self.comm)
        del buf
        m = recv.shape[0]
        gs, ge = self._i32(m), self._i32(m)
        self._sync()
        if m:
            self.ctx.deinterleave(m, 2, recv.data_ptr(), gs.data_ptr(), ge.data_ptr())
        self._sync()
        self.moved += sum(rc) - rc[self.rank]
        return m, gs, ge

    def bitset(self, n, d_contig, d_start, d_end):
        """this shard's bitset of one set, from this rank's slice of its rows"""
        ctx, sp = self.ctx, self.space
        if self.world == 1:
            return ctx.bitset_from_device(sp, n, d_contig, d_start, d_end)
        self._ensure_splits([(n, d_contig, d_start, d_end)])
        m, rgs, rge = self.shard_rows(n, d_contig, d_start, d_end)
        return ctx.bitset_from_global(sp, self.lo, self.hi, m, rgs.data_ptr(), rge.data_ptr())

    def _route_clipped(self, n, d_contig, d_start, d_end):
        """one set's rows, clipped to the shards they overlap and grouped by
        shard: an interleaved [pieces, 2] (gs, ge) int32 device tensor (the
        all_to_all send buffer as it stands) and the per-shard counts"""
        ctx, sp = self.ctx, self.space
        cap = n + 4096
        buf = torch.empty((cap, 2), dtype=torch.int32, device=self.dev)
        counts = ctx.route_rows_interleaved(sp, n, d_contig, d_start, d_end, self.splits, 2,
                                            buf.data_ptr(), clip=True, cap=cap)
        if sum(counts) > cap:  # many rows cross shard bounds: exact size
            cap = sum(counts)
            buf = torch.empty((cap, 2), dtype=torch.int32, device=self.dev)
            counts = ctx.route_rows_interleaved(sp, n, d_contig, d_start, d_end, self.splits, 2,
                                                buf.data_ptr(), clip=True, cap=cap)
        return buf, counts

    def and_bitset(self, inputs):
        """this shard's AND of k sets in one fused paint per 16
        (lime_bitset_and_from_device / _from_global): no per-set bitsets.
        The k sets' rows move in ONE packed all_to_all (dist.exchange_sets)."""
        ctx, sp = self.ctx, self.space
        if self.world == 1:
            return ctx.bitset_and_from_device(sp, inputs)
        self._ensure_splits(inputs)
        routed = [self._route_clipped(*x) for x in inputs]
        self._sync()
        got = ld.exchange_sets_rows([b for b, _ in routed], [c for _, c in routed], self.group,
                                    self.comm)
        del routed
        self._sync()
        self.moved += sum(x for _, _, x in got)
        # each rank's slice of each set straight into the set's columns (one
        # device pass per slice, no concatenation)
        cols = []
        for slices, m, _ in got:
            gs, ge = self._i32(m), self._i32(m)
            at = 0
            for t in slices:
                k = t.shape[0]
                if k:
                    ctx.deinterleave(k, 2, t.data_ptr(), gs[at:].data_ptr(), ge[at:].data_ptr())
                at += k
            cols.append((m, gs, ge))
        res = ctx.bitset_and_from_global(sp, self.lo, self.hi,
                                         [(m, gs.data_ptr(), ge.data_ptr()) for m, gs, ge in cols])
        self._sync()  # (the received slices stay referenced until the engine read them)
        del got
        return res

    def run(self, inputs, gather=False, op="and"):
        """inputs: [(n, d_contig, d_start, d_end)] per set (this rank's rows,
        device pointers); op "and" (k sets: C5), "not" (1 set: complement of
        its union against the genome), "andnot" (2 sets: per-base
        difference).  Returns a dict: the shard's result (global
        coordinates), the carry (drop_first, new_last_end), the total run
        count of the unsharded result and, with gather=True, every run as an
        int64 [m, 2] tensor (global start, end) in order."""
        self._ensure_splits(inputs)
        if op == "and":
            bits = [self.and_bitset(inputs)]
            res = self.ctx.bitset_runs(0, bits[0])
        elif op == "not":
            bits = [self.bitset(*inputs[0])]
            res = self.ctx.bitset_runs(1, bits[0])
        elif op == "andnot":
            bits = [self.bitset(*x) for x in inputs[:2]]
            res = self.ctx.bitset_runs(3, bits[0], bits[1])
        else:
            raise ValueError(f"unknown op {op}")
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


ShardedAnd = ShardedBitset  # C5's name for it
