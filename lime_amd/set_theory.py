"""Host mirror of lime-core's operator API over the MI355X engine.

Same class names, argument meaning and error behaviour as
lime-core/src/main/scala/org/bdgenomics/lime/set_theory/:

    DistributedIntersection(leftRdd, rightRdd, partitionMap, threshold=0).compute()
        -> [(ReferenceRegion, (T, U))]             Intersection.scala:45-69
    DistributedMerge(rddToCompute, partitionMap, threshold=0).compute()
        -> [(ReferenceRegion, [T])]                Merge.scala:34-36
    DistributedSubtract(leftRdd, rightRdd, partitionMap, threshold=0).compute()
        -> [(ReferenceRegion, (T, U or None))]     Subtract.scala:78-116
    DistributedComplement(rddToCompute, partitionMap, referenceNameBounds,
                          threshold=0).compute()
        -> [(ReferenceRegion, [])]                 Complement.scala:131-134
    DistributedWindow(leftRdd, rightRdd, partitionMap, threshold=1000).compute()
        -> [(ReferenceRegion, (T, U))]             Window.scala:71-95
    SingleClosest / SingleClosestSingleOverlap(leftRdd, rightRdd,
                  partitionMap).compute()
        -> [(ReferenceRegion, (T, U))]             Closest.scala:34-268
    UnstrandedCluster / StrandedCluster / ...WithMinimumOverlap(rddToCompute,
                          partitionMap, threshold=0).compute()
        -> [(ReferenceRegion, [T])]                Cluster.scala:38-121

An "RDD" here is any iterable of (ReferenceRegion, value) pairs held on the
host.  `partitionMap` is accepted for signature parity and ignored: the
engine is partition-free and its output equals the reference's single-
partition (P = 1) execution, in the same emission order (SURVEY.md
Appendix A).  Strand: for the pairwise operators rows are grouped by strand
and each group runs through the engine separately, which is exactly
ReferenceRegion.overlaps' strand equality; merge and the stranded clusters
run mixed strands as one stranded set (a run breaks at every strand change
of the (start, end, strand) order, as the reference fold does); complement
ignores strand (its gap regions carry none).
"""
from collections import namedtuple

import numpy as np

from . import _ffi
from .engine import Context, Space

STRANDS = ("INDEPENDENT", "FORWARD", "REVERSE", "UNKNOWN")  # engine codes 0..3
# RegionOrdering compares bdg-formats' Strand enum ordinals
_STRAND_ORD = {"FORWARD": 0, "REVERSE": 1, "INDEPENDENT": 2, "UNKNOWN": 3}
_STRAND_CODE = {s: i for i, s in enumerate(STRANDS)}


class ReferenceRegion(namedtuple("ReferenceRegion", "referenceName start end strand")):
    """ADAM ReferenceRegion (0-based half-open), strand as a name."""
    __slots__ = ()

    def __new__(cls, referenceName, start, end, strand="INDEPENDENT"):
        if start < 0 or end < start:
            raise ValueError(f"invalid region {referenceName}:{start}-{end}")
        return super().__new__(cls, referenceName, int(start), int(end), strand)

    @classmethod
    def unstranded(cls, name, start, end):
        return cls(name, start, end, "INDEPENDENT")


class NoSuchElementException(KeyError):
    """Raised where the reference throws java.util.NoSuchElementException."""


_CTX = None


def default_context():
    global _CTX
    if _CTX is None:
        _CTX = Context(0)
    return _CTX


def _rows(rdd):
    rdd = list(rdd)
    regions = [r for r, _ in rdd]
    values = [v for _, v in rdd]
    return regions, values


# an engine space holds u32 global coordinates: its span sum(len + 1) must
# not exceed 2^32 - 1 (lime_space_create).  Larger genomes are cut into
# several spaces (tests lower the cap to exercise the cut).
SPAN_CAP = 0xFFFFFFFF


class _Genome:
    """The contigs, in RegionOrdering (Java string order of the names), cut
    into consecutive groups whose spans fit one engine space each.  Every
    operator but closest is contig-local and runs group by group; closest
    chains its sweep's liveness from group to group
    (lime_closest_count_chained).  A genome below 2^32 is one group."""

    def __init__(self, names, lengths):
        # (engine.Space orders its contigs the same way)
        order = sorted(range(len(names)), key=lambda i: _java_key(names[i]))
        cap = SPAN_CAP
        self.spaces, self.group = [], {}
        cn, cl, span = [], [], 0
        for i in order:
            n, ln = names[i], int(lengths[i])
            if ln + 1 > cap:
                raise _ffi.LimeError(2, f"contig {n} is longer than a space can hold "
                                        f"({cap - 1})")  # LIME_ERR_RANGE
            if cn and span + ln + 1 > cap:
                self.spaces.append(Space(cn, cl))
                cn, cl, span = [], [], 0
            self.group[n] = len(self.spaces)
            cn.append(n)
            cl.append(ln)
            span += ln + 1
        if cn or not self.spaces:
            self.spaces.append(Space(cn, cl))

    def split(self, regions, rows):
        """rows (indices into regions) per group, in their given order"""
        out = [[] for _ in self.spaces]
        for i in rows:
            try:
                out[self.group[regions[i].referenceName]].append(i)
            except KeyError as e:
                raise NoSuchElementException(f"key not found: {e.args[0]}") from None
        return out


def _space_for(*region_lists, bounds=None):
    if bounds is not None:
        return _Genome(list(bounds.keys()), [b.end for b in bounds.values()])
    ext = {}
    for regs in region_lists:
        for r in regs:
            ext[r.referenceName] = max(ext.get(r.referenceName, 0), r.end)
    return _Genome(list(ext.keys()), list(ext.values()))


def _arrays(space, regions, rows):
    try:
        c = np.array([space.index[regions[i].referenceName] for i in rows], dtype=np.int32)
    except KeyError as e:
        raise NoSuchElementException(f"key not found: {e.args[0]}") from None
    s = np.array([regions[i].start for i in rows], dtype=np.int64)
    e = np.array([regions[i].end for i in rows], dtype=np.int64)
    return c, s, e


def _strand_groups(regions):
    groups = {}
    for i, r in enumerate(regions):
        groups.setdefault(r.strand, []).append(i)
    return groups


def _sorted_rank(regions):
    """Rank of every row in RegionOrdering (name, start, end, strand), stable."""
    keys = sorted(range(len(regions)), key=lambda i: (
        _java_key(regions[i].referenceName), regions[i].start, regions[i].end,
        _STRAND_ORD.get(regions[i].strand, 4), i))
    rank = np.empty(len(regions), dtype=np.int64)
    rank[keys] = np.arange(len(regions))
    return rank


def _java_key(name):
    return name.encode("utf-16-be")


class _Op:
    def __init__(self, ctx=None):
        self.ctx = ctx or default_context()


class DistributedIntersection(_Op):
    def __init__(self, leftRdd, rightRdd, partitionMap=None, threshold=0, ctx=None):
        super().__init__(ctx)
        self.left, self.right = list(leftRdd), list(rightRdd)
        self.partitionMap, self.threshold = partitionMap, int(threshold)

    def compute(self):
        lr, lv = _rows(self.left)
        rr, rv = _rows(self.right)
        genome = _space_for(lr, rr)
        lg, rg = _strand_groups(lr), _strand_groups(rr)
        out = []
        for strand, lrows_all in lg.items():
            rrows_all = rg.get(strand)
            if not rrows_all:
                continue
            for space, lrows, rrows in zip(genome.spaces, genome.split(lr, lrows_all),
                                           genome.split(rr, rrows_all)):
                if not lrows or not rrows:
                    continue
                A = self.ctx.set_from_host(space, *_arrays(space, lr, lrows))
                B = self.ctx.set_from_host(space, *_arrays(space, rr, rrows))
                plan = self.ctx.intersect(A, B, self.threshold)
                pairs = plan.fill_host()
                for p in pairs:
                    a = lrows[p["a_row"]]
                    b = rrows[p["b_row"]]
                    out.append((a, b, int(p["start"]), int(p["end"])))
                plan.close()
                A.close()
                B.close()
        # reference emission order (P = 1): left in sorted order, then cache
        # (= sorted right) order -- SetTheory.scala:181-186
        lrank, rrank = _sorted_rank(lr), _sorted_rank(rr)
        out.sort(key=lambda t: (lrank[t[0]], rrank[t[1]]))
        return [(ReferenceRegion(lr[a].referenceName, s, e, lr[a].strand), (lv[a], rv[b]))
                for a, b, s, e in out]


class DistributedWindow(_Op):
    """Window.scala:71-95: (leftRegion, (T, U)) for every right row nearby
    (ADAM isNearby, default distance 1000) each left row."""

    def __init__(self, leftRdd, rightRdd, partitionMap=None, threshold=1000, ctx=None):
        super().__init__(ctx)
        self.left, self.right = list(leftRdd), list(rightRdd)
        self.partitionMap, self.threshold = partitionMap, int(threshold)

    def compute(self):
        lr, lv = _rows(self.left)
        rr, rv = _rows(self.right)
        genome = _space_for(lr, rr)
        lg, rg = _strand_groups(lr), _strand_groups(rr)
        out = []
        for strand, lrows_all in lg.items():
            rrows_all = rg.get(strand)
            if not rrows_all:
                continue
            for space, lrows, rrows in zip(genome.spaces, genome.split(lr, lrows_all),
                                           genome.split(rr, rrows_all)):
                if not lrows or not rrows:
                    continue
                A = self.ctx.set_from_host(space, *_arrays(space, lr, lrows))
                B = self.ctx.set_from_host(space, *_arrays(space, rr, rrows))
                plan = self.ctx.window(A, B, self.threshold)
                for p in plan.fill_host():
                    out.append((lrows[p["a_row"]], rrows[p["b_row"]]))
                plan.close()
                A.close()
                B.close()
        # P = 1 emission order: left in sorted order, then cache order
        lrank, rrank = _sorted_rank(lr), _sorted_rank(rr)
        out.sort(key=lambda t: (lrank[t[0]], rrank[t[1]]))
        return [(lr[a], (lv[a], rv[b])) for a, b in out]


class SingleClosest(_Op):
    """Closest.scala:34-214 (the CLI's closest): for each left row, in
    RegionOrdering, the cached right rows at the same unstrandedDistance as
    the sweep's currentClosest -> [(leftRegion, (T, U))].  One stranded set
    per side (the order includes strand; the distance ignores it), run as the
    reference's sweep runs on one partition."""

    MODE = 0

    def __init__(self, leftRdd, rightRdd, partitionMap=None, threshold=0, ctx=None):
        super().__init__(ctx)
        self.left, self.right = list(leftRdd), list(rightRdd)
        self.partitionMap, self.threshold = partitionMap, int(threshold)

    def compute(self):
        lr, lv = _rows(self.left)
        rr, rv = _rows(self.right)
        genome = _space_for(lr, rr)
        codes = lambda regs, rows: np.array([_STRAND_CODE[regs[i].strand] for i in rows],
                                            np.int8)
        out, live = [], True
        # one space after the other, the sweep's liveness carried across
        for space, lrows, rrows in zip(genome.spaces, genome.split(lr, range(len(lr))),
                                       genome.split(rr, range(len(rr)))):
            A = self.ctx.set_from_host_stranded(space, *_arrays(space, lr, lrows),
                                                codes(lr, lrows))
            B = self.ctx.set_from_host_stranded(space, *_arrays(space, rr, rrows),
                                                codes(rr, rrows))
            plan, live = self.ctx.closest_chained(A, B, self.MODE, live)
            out += [(lr[lrows[p["a_row"]]], (lv[lrows[p["a_row"]]], rv[rrows[p["b_row"]]]))
                    for p in plan.fill_host()]
            plan.close()
            A.close()
            B.close()
        return out


class SingleClosestSingleOverlap(SingleClosest):
    """Closest.scala:216-268: SingleClosest whose advance and prune also
    compare covered lengths (the suite's second variant)."""
    MODE = 1


class DistributedSubtract(_Op):
    def __init__(self, leftRdd, rightRdd, partitionMap=None, threshold=0, ctx=None,
                 mode=_ffi.SUBTRACT_LIME):
        super().__init__(ctx)
        self.left, self.right = list(leftRdd), list(rightRdd)
        self.partitionMap, self.threshold, self.mode = partitionMap, int(threshold), mode

    def compute(self):
        lr, lv = _rows(self.left)
        rr, rv = _rows(self.right)
        genome = _space_for(lr, rr)
        lg, rg = _strand_groups(lr), _strand_groups(rr)
        out = []
        for strand, lrows_all in lg.items():
            rrows_all = rg.get(strand, [])
            for space, lrows, rrows in zip(genome.spaces, genome.split(lr, lrows_all),
                                           genome.split(rr, rrows_all)):
                if not lrows:
                    continue
                A = self.ctx.set_from_host(space, *_arrays(space, lr, lrows))
                B = self.ctx.set_from_host(space, *_arrays(space, rr, rrows))
                r = self.ctx.subtract(A, B, self.threshold, self.mode)
                res = r.to_host()
                for h in (r, A, B):  # back to the pool now, not at GC
                    h.close()
                for k in range(len(res["start"])):
                    a = lrows[res["a_row"][k]]
                    b = rrows[res["b_row"][k]] if res["b_row"][k] >= 0 else None
                    out.append((a, k, b, int(res["start"][k]), int(res["end"][k])))
        lrank = _sorted_rank(lr)
        out.sort(key=lambda t: (lrank[t[0]], t[1]))  # device order within a left row
        return [(ReferenceRegion(lr[a].referenceName, s, e, lr[a].strand),
                 (lv[a], rv[b] if b is not None else None)) for a, _, b, s, e in out]


class DistributedMerge(_Op):
    def __init__(self, rddToCompute, partitionMap=None, threshold=0, ctx=None):
        super().__init__(ctx)
        self.rdd = list(rddToCompute)
        self.partitionMap, self.threshold = partitionMap, int(threshold)

    def _runs(self):
        """The SetTheory.scala:208-225 fold.  Mixed strands run as ONE
        stranded set: RegionOrdering (start, end, strand) and a run break at
        every strand change, exactly the fold's overlaps test."""
        regs, vals = _rows(self.rdd)
        genome = _space_for(regs)
        rank = _sorted_rank(regs)
        runs = []
        for space, rows in zip(genome.spaces, genome.split(regs, range(len(regs)))):
            if not rows:
                continue
            c, s, e = _arrays(space, regs, rows)
            if len({regs[i].strand for i in rows}) > 1:
                st = np.array([_STRAND_CODE.get(regs[i].strand, 0) for i in rows], dtype=np.int8)
                A = self.ctx.set_from_host_stranded(space, c, s, e, st)
            else:
                A = self.ctx.set_from_host(space, c, s, e)
            res = self.ctx.merge(A)
            h = res.to_host()
            rid = res.run_of_row(len(rows))
            members = [[] for _ in range(len(h["start"]))]
            for k in np.argsort(rank[rows], kind="stable"):
                members[rid[k]].append(rows[k])
            runs += [(ReferenceRegion(space.names[h["contig"][k]], int(h["start"][k]),
                                      int(h["end"][k]), regs[members[k][0]].strand if members[k]
                                      else "INDEPENDENT"), [vals[i] for i in members[k]])
                     for k in range(len(h["start"]))]
            res.close()
            A.close()
        return runs

    def compute(self):
        return self._runs()


class DistributedComplement(_Op):
    def __init__(self, rddToCompute, partitionMap=None, referenceNameBounds=None, threshold=0,
                 ctx=None):
        super().__init__(ctx)
        if referenceNameBounds is None:
            raise ValueError("referenceNameBounds is required")
        self.rdd = list(rddToCompute)
        self.partitionMap, self.bounds, self.threshold = partitionMap, referenceNameBounds, \
            int(threshold)

    def compute(self):
        regs, _ = _rows(self.rdd)
        genome = _space_for(bounds=self.bounds)
        out = []
        for space, rows in zip(genome.spaces, genome.split(regs, range(len(regs)))):
            A = self.ctx.set_from_host(space, *_arrays(space, regs, rows))
            h = self.ctx.complement(space, A).to_host()
            out += [(ReferenceRegion(space.names[h["contig"][k]], int(h["start"][k]),
                                     int(h["end"][k])), []) for k in range(len(h["start"]))]
            A.close()
        return out


class _Cluster(_Op):
    """Cluster.scala:8-36: the SetTheory.scala:208-225 fold of Merge, keyed by
    the cluster's FIRST member region (postProcess :33-35) instead of the
    hull.  localCompute passes no threshold to `condition` (quirk Q6), so at
    P = 1 every variant is the strict-overlap fold: covers (strand-blind) for
    the Unstranded variants, overlaps (equal strands) for the Stranded ones."""
    STRANDED = False

    def __init__(self, rddToCompute, partitionMap=None, threshold=0, ctx=None):
        super().__init__(ctx)
        self.rdd = list(rddToCompute)
        self.partitionMap, self.threshold = partitionMap, int(threshold)

    def compute(self):
        regs, vals = _rows(self.rdd)
        genome = _space_for(regs)
        rank = _sorted_rank(regs)
        out = []
        for space, rows in zip(genome.spaces, genome.split(regs, range(len(regs)))):
            if not rows:
                continue
            c, s, e = _arrays(space, regs, rows)
            if self.STRANDED and len({regs[i].strand for i in rows}) > 1:
                st = np.array([_STRAND_CODE.get(regs[i].strand, 0) for i in rows], dtype=np.int8)
                A = self.ctx.set_from_host_stranded(space, c, s, e, st)
            else:
                A = self.ctx.set_from_host(space, c, s, e)
            res = self.ctx.merge(A)
            rid = res.run_of_row(len(rows))
            members = [[] for _ in range(res.n)]
            for k in np.argsort(rank[rows], kind="stable"):
                members[rid[k]].append(rows[k])
            res.close()
            A.close()
            # fold order = run order = order of each cluster's first member
            out += [(regs[m[0]], [vals[i] for i in m]) for m in members if m]
        return out


class UnstrandedCluster(_Cluster):
    """Cluster.scala:38-57 (condition: covers, strand-blind)."""


class UnstrandedClusterWithMinimumOverlap(_Cluster):
    """Cluster.scala:80-100 (coversBy >= threshold; Q6: threshold 0 in the fold)."""


class StrandedCluster(_Cluster):
    """Cluster.scala:59-78 (condition: overlaps, equal strands)."""
    STRANDED = True


class StrandedClusterWithMinimumOverlap(_Cluster):
    """Cluster.scala:102-121 (overlapsBy >= threshold; Q6: threshold 0 in the fold)."""
    STRANDED = True
