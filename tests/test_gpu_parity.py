"""Parity of the HIP engine (through the C-ABI) with the CPU oracle and the
reference's golden vectors.  Integer work: every comparison is bit-exact,
as sorted lists."""
import os

import numpy as np
import pytest

from lime_amd import LimeError, Space, SUBTRACT_LIME, SUBTRACT_SET, synth
from lime_amd.set_theory import (DistributedComplement, DistributedIntersection,
                                 DistributedMerge, DistributedSubtract, DistributedWindow,
                                 NoSuchElementException, ReferenceRegion, StrandedCluster,
                                 UnstrandedCluster, UnstrandedClusterWithMinimumOverlap)
from oracle import oracle
from tests.util import (GOLDEN, as_sorted_tuples, expected, random_sets, read_bed_py,
                        read_genome_py)

pytestmark = pytest.mark.gpu


def keyed(name):
    chrom, s, e, nm = read_bed_py(os.path.join(GOLDEN, name))
    return [(ReferenceRegion.unstranded(c, a, b), n) for c, a, b, n in zip(chrom, s, e, nm)]


def rr(triples):
    return [ReferenceRegion(c, s, e) for c, s, e in triples]


# ------------------------------------------------- the reference's own suites
def test_intersection_suite(ctx):
    # IntersectionSuite.scala:8-26 (full 7-pair truth; the suite's zip pins 5)
    out = DistributedIntersection(keyed("intersect_with_overlap_00.bed"),
                                  keyed("intersect_with_overlap_01.bed"), None, ctx=ctx).compute()
    regs = [r for r, _ in out]
    assert regs[:5] == rr(expected()["intersection_prefix"])
    assert regs == rr(expected()["intersection_full"])
    assert out[0][1] == ("CpG:_30", "CpG:_116")


def test_subtract_suite(ctx):
    # SubtractSuite.scala:8-40
    out = DistributedSubtract(keyed("intersect_with_overlap_00.bed"),
                              keyed("intersect_with_overlap_01.bed"), None, ctx=ctx).compute()
    assert [r for r, _ in out] == rr(expected()["subtract"])
    assert sum(v[1] is None for _, v in out) == 17


def test_merge_suite(ctx):
    # MergeSuite.scala:12-19
    out = DistributedMerge(keyed("cpg_20merge.bed"), None, ctx=ctx).compute()
    assert len(out) == expected()["merge_count"]
    assert out[0][0] == ReferenceRegion("chr1", 28735, 30000)
    assert len(out[0][1]) == 20


def test_complement_suite(ctx):
    # ComplementSuite.scala:8-115
    names, lens = read_genome_py(os.path.join(GOLDEN, "genome.txt"))
    bounds = {n: ReferenceRegion(n, 0, l) for n, l in zip(names, lens)}
    out = DistributedComplement(keyed("cpg_20merge.bed"), None, bounds, ctx=ctx).compute()
    assert [r for r, _ in out] == rr(expected()["complement"])


def test_window_suite(ctx):
    # WindowSuite.scala:8-34 (default distance 1000): all 10 bedtools pairs
    out = DistributedWindow(keyed("intersect_with_overlap_00.bed"),
                            keyed("window_with_overlap_01.bed"), None, ctx=ctx).compute()
    got = [[[r.referenceName, r.start, r.end]] for r, _ in out]
    assert [g[0] for g in got] == [p[0] for p in expected()["window"]]
    right = {n: (c, a, b) for c, a, b, n in zip(*read_bed_py(
        os.path.join(GOLDEN, "window_with_overlap_01.bed")))}
    assert [list(right[v[1]]) for _, v in out] == [p[1] for p in expected()["window"]]


def test_cluster_suite(ctx):
    # ClusterSuite.scala:8-16: cpg_20merge.bed clusters into one
    rows = keyed("cpg_20merge.bed")
    out = UnstrandedCluster(rows, None, ctx=ctx).compute()
    assert len(out) == 1
    first = min(rows, key=lambda kv: (kv[0].start, kv[0].end))
    assert out[0][0] == first[0]  # keyed by the first member, not the hull
    assert len(out[0][1]) == 20


_ORD = {"FORWARD": 0, "REVERSE": 1, "INDEPENDENT": 2, "UNKNOWN": 3}


def _fold_clusters(regs, stranded):
    """Merge.scala / Cluster.scala fold restated on the rows in RegionOrdering
    (name, start, end, strand enum ordinal): a new cluster whenever the row
    does not strictly overlap the running hull or, stranded, has another
    strand; returns member index lists in fold order."""
    order = sorted(range(len(regs)), key=lambda i: (regs[i].referenceName, regs[i].start,
                                                    regs[i].end, _ORD[regs[i].strand], i))
    out, cur, hull = [], [], None
    for i in order:
        r = regs[i]
        if (cur and r.referenceName == hull[0] and r.start < hull[2] and r.end > hull[1]
                and (not stranded or r.strand == hull[3])):
            cur.append(i)
            hull = (hull[0], min(hull[1], r.start), max(hull[2], r.end), hull[3])
        else:
            if cur:
                out.append(cur)
            cur, hull = [i], (r.referenceName, r.start, r.end, r.strand)
    if cur:
        out.append(cur)
    return out


@pytest.mark.parametrize("seed", [81, 82, 83])
def test_stranded_merge_parity(ctx, seed):
    # the reference fold with mixed strands (the CLI keys stranded regions):
    # RegionOrdering (start, end, strand) and a run break at every strand
    # change; engine stranded set == C oracle == restated fold
    rng = np.random.default_rng(seed)
    (c, s0, e0), _ = random_sets(rng, 4000, 1, n_contigs=3, contig_len=20000, max_len=400,
                                 zero_frac=0.05, dup_frac=0.1, book_frac=0.05)
    codes = rng.integers(0, 4, len(c)).astype(np.int8)
    # ties: copies of rows with another strand
    k = rng.random(len(c)) < 0.1
    src = rng.integers(0, len(c), len(c))
    c[k], s0[k], e0[k] = c[src[k]], s0[src[k]], e0[src[k]]
    sp = space_for(3, 20000)
    A = ctx.set_from_host_stranded(sp, c, s0, e0, codes)
    res = ctx.merge(A)
    got = res.to_host()
    rid = res.run_of_row(len(c))
    exp = oracle.merge((c, s0, e0, codes))
    assert got["start"].tolist() == exp["start"].tolist()
    assert got["end"].tolist() == exp["end"].tolist()
    assert got["contig"].tolist() == exp["contig"].tolist()
    assert rid.tolist() == exp["run_of_row"].tolist()
    # the operator mirror on ReferenceRegions, against the restated fold
    names = ["INDEPENDENT", "FORWARD", "REVERSE", "UNKNOWN"]
    regs = [ReferenceRegion(NAMES[ci], int(a), int(b), names[st]) for ci, a, b, st in
            zip(c, s0, e0, codes)]
    out = DistributedMerge([(r, i) for i, r in enumerate(regs)], None, ctx=ctx).compute()
    fold = _fold_clusters(regs, True)
    assert [v for _, v in out] == fold
    assert [k.strand for k, _ in out] == [regs[m[0]].strand for m in fold]


@pytest.mark.parametrize("seed", [71, 72])
def test_cluster_parity(ctx, seed):
    rng = np.random.default_rng(seed)
    (c, s0, e0), _ = random_sets(rng, 3000, 1, n_contigs=3, contig_len=40000, max_len=300,
                                 zero_frac=0.05, dup_frac=0.05, book_frac=0.1)
    strands = rng.choice(["FORWARD", "REVERSE"], len(c))
    regs = [ReferenceRegion(NAMES[ci], int(a), int(b), st) for ci, a, b, st in
            zip(c, s0, e0, strands)]
    rows = [(r, i) for i, r in enumerate(regs)]
    for op, stranded in ((UnstrandedCluster, False), (UnstrandedClusterWithMinimumOverlap, False),
                         (StrandedCluster, True)):
        got = op(rows, None, ctx=ctx).compute()
        exp = _fold_clusters(regs, stranded)
        assert [(k, v) for k, v in got] == [(regs[m[0]], m) for m in exp]


def test_complement_missing_contig_raises(ctx):
    bounds = {"chr2": ReferenceRegion("chr2", 0, 100)}
    with pytest.raises(NoSuchElementException):
        DistributedComplement(keyed("cpg_20merge.bed"), None, bounds, ctx=ctx).compute()


def test_stranded_intersection(ctx):
    # ReferenceRegion.overlaps requires equal strands (the CLI keys stranded)
    L = [(ReferenceRegion("chr1", 0, 100, "FORWARD"), "a"),
         (ReferenceRegion("chr1", 0, 100, "REVERSE"), "b")]
    R = [(ReferenceRegion("chr1", 50, 60, "FORWARD"), "x")]
    out = DistributedIntersection(L, R, None, ctx=ctx).compute()
    assert out == [(ReferenceRegion("chr1", 50, 60, "FORWARD"), ("a", "x"))]


# ----------------------------------------------------- randomised parity
NAMES = [f"c{i:02d}" for i in range(4)]


def space_for(n_contigs, contig_len):
    return Space(NAMES[:n_contigs], [contig_len] * n_contigs)


def engine_pairs(ctx, sp, A, B, t):
    a = ctx.set_from_host(sp, *A)
    b = ctx.set_from_host(sp, *B)
    plan = ctx.intersect(a, b, t)
    p = plan.fill_host()
    # contig of a pair = contig of its left row
    return {"contig": A[0][p["a_row"]], "start": p["start"], "end": p["end"],
            "a_row": p["a_row"], "b_row": p["b_row"]}, plan


CASES = [(1, 0, 0.0, 0.0), (2, 0, 0.1, 0.1), (3, 25, 0.0, 0.0), (4, -3, 0.2, 0.1),
         (5, 1, 0.1, 0.0), (6, 120, 0.05, 0.2), (7, 0, 0.0, 0.3)]


@pytest.mark.parametrize("seed,t,zero,book", CASES)
def test_intersect_parity(ctx, seed, t, zero, book):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 3000, 2500, n_contigs=3, contig_len=30000, max_len=400,
                       zero_frac=zero, dup_frac=0.05, book_frac=book)
    sp = space_for(3, 30000)
    got, plan = engine_pairs(ctx, sp, A, B, t)
    exp = oracle.intersect(A, B, t)
    assert plan.n == len(exp["start"])
    assert as_sorted_tuples(got) == as_sorted_tuples(exp)
    # device checksum kernel == checksum of the materialised pairs == oracle
    assert plan.checksum() == oracle.checksum_pairs(got) == oracle.checksum_pairs(exp)


# Deep pile-ups: partner windows of a 1024-owner tile beyond the fill
# kernel's LDS window (1792 rows) take the global-memory path, and windows
# just below it fill the whole register-prefetched LDS window.
@pytest.mark.parametrize("seed,n,contig_len,max_len", [(41, 5000, 60000, 7500),
                                                         (42, 6000, 12000, 3000),
                                                         (43, 3000, 5000, 4000)])
def test_intersect_deep_windows(ctx, seed, n, contig_len, max_len):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, n, n, n_contigs=1, contig_len=contig_len, max_len=max_len,
                       zero_frac=0.02, dup_frac=0.05)
    sp = space_for(1, contig_len)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    plan = ctx.intersect(a, b)
    exp = oracle.intersect(A, B)
    assert plan.n == len(exp["start"])
    want = oracle.checksum_pairs(exp)
    assert oracle.checksum_pairs(plan.fill_host()) == want
    assert plan.checksum() == want


# Fill windows of odd sizes and offsets ([first, first + count), records
# of one owner split across windows): their concatenation is the whole fill,
# for a sparse plan (the thread-per-owner fill, ~4 pairs per owner) and a
# dense one (k_fill)
@pytest.mark.parametrize("seed,max_len", [(81, 60), (82, 3000)])
def test_intersect_fill_windows(ctx, seed, max_len):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 6000, 5000, n_contigs=2, contig_len=40000, max_len=max_len,
                       zero_frac=0.02, dup_frac=0.05)
    sp = space_for(2, 40000)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    plan = ctx.intersect(a, b)
    exp = oracle.intersect(A, B)
    assert plan.n == len(exp["start"])
    whole = plan.fill_host()
    parts, f = [], 0
    for k in [1, 777, 4096, 63, 100000]:
        k = min(k, plan.n - f)
        if k <= 0:
            break
        parts.append(plan.fill_host(f, k))
        f += k
    if f < plan.n:
        parts.append(plan.fill_host(f, plan.n - f))
    cat = np.concatenate(parts)
    for key in whole.dtype.names:
        assert cat[key].tolist() == whole[key].tolist()
    want = oracle.checksum_pairs(exp)
    assert oracle.checksum_pairs(whole) == want
    assert plan.checksum() == want


# One plan whose tiles differ in density: a dense contig (the fill finds a
# tile's ranges in its LDS window itself, >= 32 pairs per owner) next to a
# sparse one (k_count's staged ranges), zero-width partners (the search skips
# them at a.s) and a threshold (its hi keys, not filtered: no row narrower)
@pytest.mark.parametrize("seed,t", [(71, 0), (72, 20), (73, -5)])
def test_intersect_mixed_density(ctx, seed, t):
    rng = np.random.default_rng(seed)

    def one(n):
        c = (rng.random(n) < 0.5).astype(np.int32)
        lo = max(t, 1)
        s = np.where(c == 0, rng.integers(0, 37000, n), rng.integers(0, 399000, n))
        l = np.where(c == 0, rng.integers(lo, 3000, n), rng.integers(lo, 60, n))
        if t <= 0:
            l[rng.random(n) < 0.03] = 0
        return c, s.astype(np.int64), s.astype(np.int64) + l.astype(np.int64)

    A, B = one(8000), one(8000)
    sp = Space(["c0", "c1"], [40000, 400000])
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    plan = ctx.intersect(a, b, t)
    exp = oracle.intersect(A, B, t)
    assert plan.n == len(exp["start"])
    want = oracle.checksum_pairs(exp)
    assert oracle.checksum_pairs(plan.fill_host()) == want
    assert plan.checksum() == want


@pytest.mark.parametrize("seed,d", [(61, 0), (62, 1), (63, 7), (64, 150), (65, 1000),
                                    (66, 40000)])
def test_window_parity(ctx, seed, d):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 2500, 2000, n_contigs=3, contig_len=30000, max_len=400,
                       zero_frac=0.1, dup_frac=0.05, book_frac=0.1)
    # contig-edge rows: zero-width and short rows at both ends of every contig
    for X in (A, B):
        k = len(X[1])
        for i, (c, s0, l) in enumerate([(0, 0, 0), (0, 0, 3), (1, 0, 0), (1, 30000, 0),
                                        (2, 29990, 10), (0, 30000, 0), (2, 0, 0)]):
            X[0][k - 1 - i], X[1][k - 1 - i], X[2][k - 1 - i] = c, s0, s0 + l
    sp = space_for(3, 30000)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    plan = ctx.window(a, b, d)
    exp = oracle.window(A, B, d)
    assert plan.n == len(exp["start"])
    p = plan.fill_host()
    got = {"contig": A[0][p["a_row"]], "start": p["start"], "end": p["end"],
           "a_row": p["a_row"], "b_row": p["b_row"]}
    assert as_sorted_tuples(got) == as_sorted_tuples(exp)
    assert plan.checksum() == oracle.checksum_pairs(exp)


@pytest.mark.parametrize("seed,zero,book", [(11, 0.0, 0.0), (12, 0.1, 0.1), (13, 0.3, 0.3)])
def test_merge_parity(ctx, seed, zero, book):
    rng = np.random.default_rng(seed)
    A, _ = random_sets(rng, 20000, 1, n_contigs=4, contig_len=60000, max_len=300,
                       zero_frac=zero, dup_frac=0.1, book_frac=book)
    sp = space_for(4, 60000)
    a = ctx.set_from_host(sp, *A)
    res = ctx.merge(a)
    h = res.to_host()
    exp = oracle.merge(A)
    assert list(h["contig"]) == list(exp["contig"])
    assert list(h["start"]) == list(exp["start"]) and list(h["end"]) == list(exp["end"])
    assert (res.run_of_row(len(A[0])) == exp["run_of_row"]).all()


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("seed,t,zero", [(21, 0, 0.0), (22, 0, 0.1), (23, 30, 0.05),
                                         (24, 1, 0.1), (25, -2, 0.0)])
def test_subtract_parity(ctx, mode, seed, t, zero):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 4000, 3000, n_contigs=3, contig_len=40000, max_len=500,
                       zero_frac=zero, dup_frac=0.05, book_frac=0.1)
    sp = space_for(3, 40000)
    res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t, mode).to_host()
    exp = oracle.subtract(A, B, t, mode)
    # exact per-left-row emission order (blocks reversed in lime mode) and the
    # block head's right row; left rows tied on start may be interleaved
    # differently (device order: start, zero-width first, row), so compare
    # after a stable grouping by left row
    og, oe = np.argsort(res["a_row"], kind="stable"), np.argsort(exp["a_row"], kind="stable")
    for k in ("contig", "start", "end", "a_row", "b_row"):
        assert list(res[k][og]) == list(exp[k][oe]), k


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("seed,t", [(26, 0), (27, 1), (28, 40), (29, -5)])
def test_subtract_long_right_intervals(ctx, mode, seed, t):
    # B holds megabase rows (gene bodies, segmental duplications) among short
    # ones: every later left row has far-back spanning hits.  The engine folds
    # all spanning hits of a row into one block found by a search (no walk
    # back over B); it must still equal the reference fold exactly.
    rng = np.random.default_rng(seed)
    L = 5_000_000
    A, B = random_sets(rng, 6000, 4000, n_contigs=2, contig_len=L, max_len=800,
                       zero_frac=0.05, dup_frac=0.05, book_frac=0.1)
    k = rng.random(len(B[0])) < 0.01  # ~40 long rows, up to 3 Mb
    B[1][k] = rng.integers(0, L // 2, k.sum())
    B[2][k] = np.minimum(B[1][k] + rng.integers(100_000, 3_000_000, k.sum()), L)
    # spanning hits sharing a start with different ends (head re-pick)
    B[1][:20], B[2][:20] = B[1][k][0], B[1][k][0] + rng.integers(1, 2_000_000, 20)
    B[0][:20] = B[0][k][0]
    sp = space_for(2, L)
    res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t, mode).to_host()
    exp = oracle.subtract(A, B, t, mode)
    og, oe = np.argsort(res["a_row"], kind="stable"), np.argsort(exp["a_row"], kind="stable")
    for key in ("contig", "start", "end", "a_row", "b_row"):
        assert list(res[key][og]) == list(exp[key][oe]), key


@pytest.mark.parametrize("seed,zero", [(31, 0.0), (32, 0.1)])
def test_complement_parity(ctx, seed, zero):
    rng = np.random.default_rng(seed)
    A, _ = random_sets(rng, 5000, 1, n_contigs=3, contig_len=50000, max_len=400,
                       zero_frac=zero, book_frac=0.1)
    lens = [50000, 50000, 50000, 777]  # last contig has no data
    sp = Space(NAMES, lens)
    res = ctx.complement(sp, ctx.set_from_host(sp, *A)).to_host()
    exp = oracle.complement(A, lens)
    for k in ("contig", "start", "end"):
        assert list(res[k]) == list(exp[k]), k


@pytest.mark.parametrize("seed,zero", [(33, 0.0), (34, 0.1), (35, None)])
def test_complement_of_merge_runs(ctx, seed, zero):
    # bench.py's C3 step: the complement from the merge's runs
    # (lime_complement_runs over [0, span)) equals lime_complement of the set
    import torch
    rng = np.random.default_rng(seed)
    if zero is None:  # no rows at all: every contig one gap
        A = (np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, np.int64))
    else:
        A, _ = random_sets(rng, 5000, 1, n_contigs=3, contig_len=50000, max_len=400,
                           zero_frac=zero, book_frac=0.1)
    lens = [50000, 50000, 50000, 777]
    sp = Space(NAMES, lens)
    S = ctx.set_from_host(sp, *A)
    mg = ctx.merge(S)
    k = mg.n
    dev = torch.device("cuda", 0)
    gs = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
    ge = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
    if k:
        mg.copy_rows_device(0, k, gs.data_ptr(), ge.data_ptr())
    got = ctx.complement_runs(sp, k, gs.data_ptr(), ge.data_ptr()).to_host()
    exp = oracle.complement(A, lens)
    for key in ("contig", "start", "end"):
        assert list(got[key]) == list(exp[key]), key


def test_sorted_set_order(ctx):
    rng = np.random.default_rng(41)
    A, _ = random_sets(rng, 50000, 1, n_contigs=4, contig_len=100000, zero_frac=0.1,
                       dup_frac=0.1)
    sp = space_for(4, 100000)
    h = ctx.set_from_host(sp, *A).to_host()
    assert sorted(h["row"]) == list(range(50000))
    c, s, e = A[0][h["row"]], A[1][h["row"]], A[2][h["row"]]
    assert (c == h["contig"]).all() and (s == h["start"]).all() and (e == h["end"]).all()
    key = list(zip(c, s, e > s, h["row"]))
    assert key == sorted(key)  # (contig, start, zero-width first), stable


def test_empty_and_errors(ctx):
    sp = space_for(2, 1000)
    z = (np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, np.int64))
    one = (np.array([1], np.int32), np.array([5]), np.array([9]))
    e = ctx.set_from_host(sp, *z)
    o = ctx.set_from_host(sp, *one)
    assert ctx.intersect(e, o).n == 0 and ctx.intersect(o, e).n == 0
    assert ctx.merge(e).n == 0
    r = ctx.subtract(o, e).to_host()
    assert list(r["start"]) == [5] and list(r["b_row"]) == [-1]
    assert ctx.subtract(e, o).n == 0
    assert ctx.complement(sp, e).n == 2
    with pytest.raises(LimeError) as ei:
        ctx.set_from_host(sp, np.array([2], np.int32), np.array([0]), np.array([1]))
    assert ei.value.code == 5
    with pytest.raises(LimeError) as ei:
        ctx.set_from_host(sp, np.array([0], np.int32), np.array([0]), np.array([1001]))
    assert ei.value.code == 2


def test_device_synth_matches_numpy(ctx):
    import torch
    sp = Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    n = 200000
    c = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    e = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.synth_uniform(sp, n, 0xA, 50, 5000, c.data_ptr(), s.data_ptr(), e.data_ptr())
    ctx.synchronize()
    ec, es, ee = synth.uniform(sp.lengths, n, 0xA, 50, 5000)
    assert (c.cpu().numpy() == ec).all()
    assert (s.cpu().numpy().view(np.uint32) == es).all()
    assert (e.cpu().numpy().view(np.uint32) == ee).all()
    ctx.synth_pileup(sp, n, 0xC, 5000, 150, 150, 600, c.data_ptr(), s.data_ptr(), e.data_ptr())
    ctx.synchronize()
    pc, ps, pe = synth.pileup(sp.lengths, n, 0xC, 5000, 150, 150, 600)
    assert (c.cpu().numpy() == pc).all() and (s.cpu().numpy().view(np.uint32) == ps).all()


def _device_set(ctx, sp, n, seed, lo, hi):
    import torch
    c = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    e = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.synth_uniform(sp, n, seed, lo, hi, c.data_ptr(), s.data_ptr(), e.data_ptr())
    return ctx.set_from_device(sp, n, c.data_ptr(), s.data_ptr(), e.data_ptr())


def test_scaled_c2_parity(ctx):
    # C2's distribution on a 1/400 genome: same depth (~82 per set), so the
    # same pairs per row; small enough for the oracle
    lens = [x // 400 for x in synth.HG38.values()]
    sp = Space(list(synth.HG38.keys()), lens)
    n = 250_000
    A = synth.uniform(sp.lengths, n, 0xA, 50, 5000)
    B = synth.uniform(sp.lengths, n, 0xB, 50, 5000)
    a = _device_set(ctx, sp, n, 0xA, 50, 5000)
    b = _device_set(ctx, sp, n, 0xB, 50, 5000)
    plan = ctx.intersect(a, b)
    exp = oracle.intersect(A, B)
    assert plan.n == len(exp["start"])
    assert plan.checksum() == oracle.checksum_pairs(exp)
    # chunked device fill (odd chunk size) reproduces the checksum
    import torch
    from lime_amd import PAIR_DTYPE
    step = 10_000_019
    tot, xr = 0, 0
    buf = torch.empty((step, 4), dtype=torch.int32, device="cuda")
    for f in range(0, plan.n, step):
        k = min(step, plan.n - f)
        plan.fill_device(f, k, buf.data_ptr())
        ctx.synchronize()
        p = buf[:k].cpu().numpy().view(np.uint32).reshape(-1).view(PAIR_DTYPE)
        s_, x_ = oracle.checksum_pairs(p)
        tot = (tot + s_) % 2**64
        xr ^= x_
    assert (tot, xr) == plan.checksum()
    mres = ctx.merge(a).to_host()
    mexp = oracle.merge(A)
    assert (mres["start"] == mexp["start"]).all() and (mres["end"] == mexp["end"]).all()


def test_full_size_c2_count_property(ctx):
    # BASELINE C2 at full size (2 x 1e8): the pair count must equal an
    # independent formula, #overlaps(a) = #{b.s < a.e} - #{b.e <= a.s},
    # evaluated per contig with numpy searchsorted
    sp = Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    n = 100_000_000
    a = _device_set(ctx, sp, n, 0xA, 50, 5000)
    b = _device_set(ctx, sp, n, 0xB, 50, 5000)
    plan = ctx.intersect(a, b)
    A = synth.uniform(sp.lengths, n, 0xA, 50, 5000)
    B = synth.uniform(sp.lengths, n, 0xB, 50, 5000)
    total = 0
    for c in range(len(sp.lengths)):
        ma, mb = A[0] == c, B[0] == c
        bs, be = np.sort(B[1][mb]), np.sort(B[2][mb])
        total += int(np.searchsorted(bs, A[2][ma], "left").sum() -
                     np.searchsorted(be, A[1][ma], "right").sum())
    assert plan.n == total
    assert 1.5e10 < plan.n < 1.75e10  # E[pairs] ~ 1.63e10


@pytest.mark.parametrize("seed,max_len", [(52, 300), (53, 700000)])
def test_bitset_from_unsorted_rows(ctx, seed, max_len):
    # binned paint from unsorted device rows == paint from the sorted set's
    # merged runs: same coverage, same runs of every op (rows up to 0.7 Mb
    # cross several 2^18-base tiles; zero-width rows paint nothing)
    import torch
    rng = np.random.default_rng(seed)
    A, _ = random_sets(rng, 30000, 1, n_contigs=3, contig_len=2_000_000, max_len=max_len,
                       zero_frac=0.05, dup_frac=0.02)
    sp = space_for(3, 2_000_000)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(np.ascontiguousarray(x).astype(np.int32)).to(dev) for x in A]
    torch.cuda.synchronize()
    bu = ctx.bitset_from_device(sp, len(A[0]), *(x.data_ptr() for x in t))
    bs = ctx.bitset(ctx.set_from_host(sp, *A))
    assert bu.popcount() == bs.popcount()
    for op in (0, 1):
        assert ctx.bitset_runs(op, bu).to_host()["start"].tolist() == \
            ctx.bitset_runs(op, bs).to_host()["start"].tolist()
    assert ctx.bitset_runs(3, bu, bs).n == 0 and ctx.bitset_runs(3, bs, bu).n == 0


@pytest.mark.parametrize("case", ["spread", "skewed"])
def test_bitset_sparse_and_skewed_bins(ctx, case):
    # unsorted rows -> bits over a 2-bin space: rows crossing the paint tiles
    # and the bins, rows past a bin piece's length field (cross list),
    # zero-width rows, and (skewed) one bin holding 5/6 of the rows
    import torch
    rng = np.random.default_rng(57 if case == "spread" else 58)
    n = 24000
    c = rng.integers(0, 3, n).astype(np.int32)
    s = rng.integers(0, 1_990_000, n)
    if case == "skewed":  # 20000 rows in contig 0's first 1 Mb: bin 0
        c[:20000] = 0
        s[:20000] = rng.integers(0, 1_000_000, 20000)
    ln = rng.integers(0, 400, n)
    long_rows = rng.random(n) < 0.02
    ln[long_rows] = rng.integers(1000, 9000, int(long_rows.sum()))
    e = np.minimum(s + ln, 2_000_000)
    A = (c, s.astype(np.int64), e.astype(np.int64))
    sp = space_for(3, 2_000_000)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(np.ascontiguousarray(x).astype(np.int32)).to(dev) for x in A]
    torch.cuda.synchronize()
    bu = ctx.bitset_from_device(sp, n, *(x.data_ptr() for x in t))
    bs = ctx.bitset(ctx.set_from_host(sp, *A))
    m = oracle.merge(A)
    assert bu.popcount() == bs.popcount() == int((m["end"] - m["start"]).sum())
    for op in (0, 1):
        got, want = ctx.bitset_runs(op, bu).to_host(), ctx.bitset_runs(op, bs).to_host()
        assert got["start"].tolist() == want["start"].tolist()
        assert got["end"].tolist() == want["end"].tolist()
    assert ctx.bitset_runs(3, bu, bs).n == 0 and ctx.bitset_runs(3, bs, bu).n == 0


def test_bitset_paths(ctx):
    rng = np.random.default_rng(51)
    A, B = random_sets(rng, 20000, 20000, n_contigs=3, contig_len=200000, max_len=300)
    sp = space_for(3, 200000)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    ba, bb = ctx.bitset(a), ctx.bitset(b)
    cov_a = sum(e - s for e, s in zip(oracle.merge(A)["end"], oracle.merge(A)["start"]))
    assert ba.popcount() == cov_a

    def coalesce(res):
        out = []
        for c, s, e in zip(res["contig"], res["start"], res["end"]):
            if out and out[-1][0] == c and out[-1][2] == s:
                out[-1][2] = e
            else:
                out.append([int(c), int(s), int(e)])
        return out
    # complement (bitset NOT) == interval complement after coalescing (A.4)
    lens = [200000] * 3
    got = ctx.bitset_runs(1, ba).to_host()
    exp = oracle.complement(A, lens)
    assert coalesce(got) == coalesce(exp)
    # difference: base-level merge(A) \ merge(B) == set-mode subtract of merged runs
    got = coalesce(ctx.bitset_runs(3, ba, bb).to_host())
    ma, mb = oracle.merge(A), oracle.merge(B)
    exp = oracle.subtract((ma["contig"], ma["start"], ma["end"]),
                          (mb["contig"], mb["start"], mb["end"]), 0, oracle.SUB_SET)
    assert got == coalesce(exp)
    # 2-way AND == merged intersection of merged operands
    got = coalesce(ctx.bitset_and([ba, bb]).to_host())
    ix = oracle.intersect((ma["contig"], ma["start"], ma["end"]),
                          (mb["contig"], mb["start"], mb["end"]))
    order = np.lexsort((ix["start"], ix["contig"]))
    exp = coalesce({k: ix[k][order] for k in ("contig", "start", "end")})
    assert got == exp


@pytest.mark.parametrize("nc", [200, 1500])
def test_contig_table_lds_and_global(ctx, nc):
    # the row passes stage the contig table in LDS up to 1024 contigs and
    # read it through the caches beyond: both branches == the oracle
    # (sort prep via set_from_host; bin count / write via bitset_from_device)
    import torch
    rng = np.random.default_rng(70 + nc)
    A, B = random_sets(rng, 40000, 30000, n_contigs=nc, contig_len=5000, max_len=400,
                       zero_frac=0.02)
    sp = Space([f"c{i}" for i in range(nc)], [5000] * nc)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    m = ctx.merge(a).to_host()
    em = oracle.merge(A)
    assert m["start"].tolist() == em["start"].tolist() and m["end"].tolist() == em["end"].tolist()
    assert ctx.intersect(a, b).n == len(oracle.intersect(A, B)["start"])
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(np.ascontiguousarray(x).astype(np.int32)).to(dev) for x in A]
    torch.cuda.synchronize()
    bu = ctx.bitset_from_device(sp, len(A[0]), *(x.data_ptr() for x in t))
    assert bu.popcount() == int((em["end"] - em["start"]).sum())
    from tests.test_gpu_configs import coalesce  # book-ended runs joined (A.4)
    comp = ctx.bitset_runs(1, bu).to_host()
    ec = oracle.complement(A, [5000] * nc)
    got = coalesce(comp["contig"], comp["start"], comp["end"])
    exp = coalesce(ec["contig"], ec["start"], ec["end"])
    for x, y in zip(got, exp):
        assert x.tolist() == y.tolist()


def _dev_rows(A):
    import torch
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(np.ascontiguousarray(x).astype(np.int32)).to(dev) for x in A]
    torch.cuda.synchronize()
    return t


@pytest.mark.parametrize("k,max_len", [(1, 300), (3, 700000), (5, 3000)])
def test_bitset_and_fused(ctx, k, max_len):
    # one fused paint of k row sets == the AND of their k bitsets (rows up to
    # 0.7 Mb leave cross pieces and wholly covered tiles)
    rng = np.random.default_rng(80 + k)
    sets = [random_sets(rng, 20000, 1, n_contigs=3, contig_len=3_000_000, max_len=max_len,
                        zero_frac=0.05, dup_frac=0.02)[0] for _ in range(k)]
    sp = space_for(3, 3_000_000)
    dev = [_dev_rows(A) for A in sets]
    fused = ctx.bitset_and_from_device(
        sp, [(len(A[0]), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr()) for A, t in
             zip(sets, dev)])
    bits = [ctx.bitset_from_device(sp, len(A[0]), *(x.data_ptr() for x in t))
            for A, t in zip(sets, dev)]
    exp = ctx.bitset_and(bits).to_host()
    got = ctx.bitset_runs(0, fused).to_host()
    assert len(exp["start"]) > 0
    for key in ("contig", "start", "end"):
        assert got[key].tolist() == exp[key].tolist()


def test_bitset_drop_bins(ctx):
    # lime_bitset_drop_bins: a bitset from rows (and the fused AND of 3 row
    # sets) paints its words and frees its binned rows; every op's runs and
    # the popcount are unchanged, and a second call is a no-op
    rng = np.random.default_rng(91)
    sets = [random_sets(rng, 20000, 1, n_contigs=3, contig_len=3_000_000, max_len=3000,
                        zero_frac=0.05, dup_frac=0.02)[0] for _ in range(3)]
    sp = space_for(3, 3_000_000)
    dev = [_dev_rows(A) for A in sets]
    rows = [(len(A[0]), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr())
            for A, t in zip(sets, dev)]
    a, b = (ctx.bitset_from_device(sp, *r) for r in rows[:2])
    fused = ctx.bitset_and_from_device(sp, rows)

    def runs(op, x, y=None):
        h = ctx.bitset_runs(op, x, y).to_host()
        return [h[k].tolist() for k in ("contig", "start", "end")]

    before = [runs(0, fused), runs(1, a), runs(2, a, b), runs(3, a, b),
              a.popcount(), fused.popcount()]
    for x in (a, b, fused):
        x.drop_bins()
    fused.drop_bins()
    after = [runs(0, fused), runs(1, a), runs(2, a, b), runs(3, a, b),
             a.popcount(), fused.popcount()]
    assert len(before[0][0]) > 0 and before[4] > 0
    assert after == before


def test_bitset_binned_runs_tile_edges(ctx):
    # bitsets from rows stay binned; an op's runs come straight from the bins
    # (k_paint_ev: per 2^19-base paint tile, events with the bit before the
    # tile taken as 0, runs crossing a tile boundary joined by k_ev_join).
    # Rows ending / starting exactly on tile boundaries, crossing them and
    # wholly covering a tile, against the words path (a bitset from the
    # sorted set: painted words) and the oracle; a dense tile past its event
    # slot falls back to the words path
    from tests.test_gpu_configs import coalesce
    T = 1 << 19
    L = 3_000_000
    rng = np.random.default_rng(97)
    sets = []
    for extra in ([(T - 100, T), (T, T + 50), (2 * T - 10, 2 * T + 10), (2 * T - 5, 3 * T + 5),
                   (4 * T, 4 * T + 1), (5 * T - 1, 5 * T)],
                  [(T - 50, T + 30), (3 * T, 3 * T + 7), (4 * T - 3, 4 * T + 3)]):
        A = random_sets(rng, 3000, 1, n_contigs=1, contig_len=L, max_len=2000, zero_frac=0.02)[0]
        A = [np.concatenate([A[0], np.zeros(len(extra), A[0].dtype)]),
             np.concatenate([A[1], np.array([a for a, _ in extra], A[1].dtype)]),
             np.concatenate([A[2], np.array([b for _, b in extra], A[2].dtype)])]
        sets.append(A)
    sp = space_for(1, L)
    binned = [ctx.bitset_from_device(sp, len(A[0]), *(x.data_ptr() for x in _dev_rows(A)))
              for A in sets]
    words = [ctx.bitset(ctx.set_from_host(sp, *A)) for A in sets]

    def runs(r):
        h = r.to_host()
        return [x.tolist() for x in coalesce(h["contig"], h["start"], h["end"])]

    ma, mb = (oracle.merge(A) for A in sets)
    for op in (0, 1, 2, 3):
        b = 1 if op >= 2 else None
        got = ctx.bitset_runs(op, binned[0], binned[b] if b else None)
        ref = ctx.bitset_runs(op, words[0], words[b] if b else None)
        mixed = ctx.bitset_runs(op, words[0], binned[b] if b else None)
        assert runs(got) == runs(ref) == runs(mixed), op
        # the fused path's runs are maximal already (no coalescing needed)
        h = got.to_host()
        assert not np.any(h["start"][1:] == h["end"][:-1])
    exp = oracle.complement(sets[0], [L])
    assert runs(ctx.bitset_runs(1, binned[0])) == [x.tolist() for x in coalesce(
        exp["contig"], exp["start"], exp["end"])]
    sub = oracle.subtract((ma["contig"], ma["start"], ma["end"]),
                          (mb["contig"], mb["start"], mb["end"]), 0, oracle.SUB_SET)
    keep = sub["end"] > sub["start"]  # (zero-width rows' runs hold no base)
    assert runs(ctx.bitset_runs(3, *binned)) == [x.tolist() for x in coalesce(
        sub["contig"][keep], sub["start"][keep], sub["end"][keep])]
    assert binned[0].popcount() == words[0].popcount() == int((ma["end"] - ma["start"]).sum())
    # the k-way AND kept binned (its runs from one k_paint_ev over both sets;
    # popcount paints its words) == the words path's a & b
    dev = [_dev_rows(A) for A in sets]
    fused = ctx.bitset_and_from_device(sp, [(len(A[0]), *(x.data_ptr() for x in t))
                                            for A, t in zip(sets, dev)])
    ref = ctx.bitset_runs(2, words[0], words[1])
    assert runs(ctx.bitset_runs(0, fused)) == runs(ref)
    pop = int((ref.to_host()["end"] - ref.to_host()["start"]).sum())
    assert fused.popcount() == pop
    nf = ctx.bitset_runs(1, fused).to_host()  # (~(a & b): the words path)
    assert int((nf["end"] - nf["start"]).sum()) == L - pop
    assert runs(ctx.bitset_runs(0, fused)) == runs(ref)  # (words painted now: same runs)
    # 3000 one-base rows two apart in tile 0: 6000 events past the 4096 slot
    n = 3000
    D = [np.zeros(n, np.int32), (10 + 2 * np.arange(n)).astype(np.uint32),
         (11 + 2 * np.arange(n)).astype(np.uint32)]
    bd = ctx.bitset_from_device(sp, n, *(x.data_ptr() for x in _dev_rows(D)))
    got = ctx.bitset_runs(0, bd).to_host()
    assert got["start"].tolist() == D[1].tolist() and got["end"].tolist() == D[2].tolist()
    assert ctx.bitset_runs(1, bd).n == n + 1

def test_bitset_and_fused_window(ctx):
    # a shard's window from global rows == the per-set window bitsets' AND
    import torch
    rng = np.random.default_rng(91)
    sp = space_for(3, 3_000_000)
    lo, hi = 64 * 20000, 7_000_000
    rows, bits = [], []
    keep = []
    for _ in range(4):
        A, _ = random_sets(rng, 20000, 1, n_contigs=3, contig_len=3_000_000, max_len=5000)
        off = sp.offsets[:3]
        gs = (off[A[0]] + A[1]).astype(np.uint32).view(np.int32)
        ge = (off[A[0]] + A[2]).astype(np.uint32).view(np.int32)
        t = [torch.from_numpy(x).cuda() for x in (gs, ge)]
        keep.append(t)
        rows.append((len(gs), t[0].data_ptr(), t[1].data_ptr()))
        bits.append(ctx.bitset_from_global(sp, lo, hi, len(gs), t[0].data_ptr(), t[1].data_ptr()))
    torch.cuda.synchronize()
    fused = ctx.bitset_and_from_global(sp, lo, hi, rows)
    assert fused.window() == bits[0].window()
    got = ctx.bitset_runs(0, fused).to_host()
    exp = ctx.bitset_and(bits).to_host()
    assert len(exp["start"]) > 0
    for key in ("contig", "start", "end"):
        assert got[key].tolist() == exp[key].tolist()


def test_bitset_cross_capacity_two_pieces_per_row(ctx):
    # rows longer than a bin piece (1023 bases) starting 10 bases before a
    # 2^19-base paint tile end leave TWO cross pieces each (bin remainder +
    # tile-crossing remainder): the cross list holds 2 n
    T = 1 << 19
    n = 60000
    j = np.arange(n) % 5 + 1
    A = (np.zeros(n, np.int32), (j * T - 10).astype(np.int64), (j * T - 10 + 2000).astype(np.int64))
    sp = space_for(1, 4_000_000)
    t = _dev_rows(A)
    cov = int((oracle.merge(A)["end"] - oracle.merge(A)["start"]).sum())
    b = ctx.bitset_from_device(sp, n, *(x.data_ptr() for x in t))
    assert b.popcount() == cov == 5 * 2000
    f = ctx.bitset_and_from_device(sp, [(n, *(x.data_ptr() for x in t))] * 2)
    assert f.popcount() == cov
    got = ctx.bitset_runs(0, f).to_host()
    em = oracle.merge(A)
    assert got["start"].tolist() == em["start"].tolist()
    assert got["end"].tolist() == em["end"].tolist()


def test_bitset_window_end_on_bin_bound(ctx):
    # window width = 2 bins (2^23 bits): rows wholly past its end clamp to
    # bit 2^23 and must land in the last tile the count pass gave them
    # (a mismatch left a tile slot unwritten)
    import torch
    rng = np.random.default_rng(93)
    sp = space_for(1, 12_000_000)
    lo, hi = 0, 1 << 23
    n = 40000
    s = rng.integers(0, 12_000_000 - 500, n)
    e = s + rng.integers(0, 500, n)
    gs = torch.from_numpy(s.astype(np.uint32).view(np.int32)).cuda()
    ge = torch.from_numpy(e.astype(np.uint32).view(np.int32)).cuda()
    torch.cuda.synchronize()
    m = oracle.merge((np.zeros(n, np.int32), s, e))
    from tests.test_gpu_configs import coalesce  # book-ended runs joined (A.4)
    cs, ce = np.clip(m["start"], lo, hi), np.clip(m["end"], lo, hi)
    keep = ce > cs
    _, xs, xe = coalesce(np.zeros(int(keep.sum())), cs[keep], ce[keep])
    assert len(xs) > 1000
    for b in (ctx.bitset_from_global(sp, lo, hi, n, gs.data_ptr(), ge.data_ptr()),
              ctx.bitset_and_from_global(sp, lo, hi, [(n, gs.data_ptr(), ge.data_ptr())])):
        got = ctx.bitset_runs(0, b).to_host()
        assert got["start"].tolist() == xs.tolist()
        assert got["end"].tolist() == xe.tolist()


@pytest.mark.parametrize("hi", [1 << 18, 3 << 18, (3 << 18) + 37, 1 << 23])
def test_bitset_runs_reaching_window_end(ctx, hi):
    # Run extraction pairs every start with an end: a run covering the
    # window's last bit closes in the tile past the last word (the extraction
    # covers one word more than the window).  Windows whose word count is an
    # exact multiple of the extraction tile (4096 words = 2^18 bits), one that
    # ends mid-word, and a 2-bin window; rows crossing the window end and a
    # row ending exactly on it; ops: bits (0), NOT within the window (1),
    # AND-NOT with an empty operand (3), the fused AND of one set.  (An
    # unpaired event raises LIME_ERR_DEVICE "odd event count" instead.)
    import torch
    from tests.test_gpu_configs import coalesce
    rng = np.random.default_rng(hi)
    sp = space_for(1, 12_000_000)
    lo = 0
    n = 30000
    s = rng.integers(0, hi, n)
    e = s + rng.integers(1, 300, n)
    s = np.concatenate([s, [hi - 100, hi - 7, hi - 1, hi - 50]])
    e = np.concatenate([e, [hi + 50, hi, hi, hi + 2000]])
    n = len(s)
    gs = torch.from_numpy(s.astype(np.uint32).view(np.int32)).cuda()
    ge = torch.from_numpy(e.astype(np.uint32).view(np.int32)).cuda()
    none = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    m = oracle.merge((np.zeros(n, np.int32), s, e))
    cs, ce = np.clip(m["start"], lo, hi), np.clip(m["end"], lo, hi)
    keep = ce > cs
    _, xs, xe = coalesce(np.zeros(int(keep.sum())), cs[keep], ce[keep])
    assert xe[-1] == hi
    # the gaps inside [lo, hi)
    gs_, ge_ = np.concatenate([[lo], xe]), np.concatenate([xs, [hi]])
    g = ge_ > gs_
    b = ctx.bitset_from_global(sp, lo, hi, n, gs.data_ptr(), ge.data_ptr())
    empty = ctx.bitset_from_global(sp, lo, hi, 0, none.data_ptr(), none.data_ptr())
    fused = ctx.bitset_and_from_global(sp, lo, hi, [(n, gs.data_ptr(), ge.data_ptr())])
    for got, (es, ee) in ((ctx.bitset_runs(0, b), (xs, xe)), (ctx.bitset_runs(1, b), (gs_[g], ge_[g])),
                          (ctx.bitset_runs(3, b, empty), (xs, xe)),
                          (ctx.bitset_runs(0, fused), (xs, xe))):
        h = got.to_host()
        assert h["start"].tolist() == es.tolist()
        assert h["end"].tolist() == ee.tolist()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_set_theory_genome_cut_into_spaces(ctx, monkeypatch, seed):
    # a genome whose span exceeds one engine space (u32 coordinates: >= 2^32)
    # is cut into consecutive spaces; lowering the cap cuts a small genome
    # the same way.  Every operator must return exactly its one-space result
    # (closest chains its sweep liveness across the cut)
    import lime_amd.set_theory as st
    rng = np.random.default_rng(300 + seed)
    names = [f"chr{i}" for i in (1, 2, 3, 10, 11, 20, 7)]
    lens = {n: int(rng.integers(5000, 20000)) for n in names}
    only_left, only_right = names[1], names[4]

    def rdd(n, side):
        out = []
        for i in range(n):
            c = names[int(rng.integers(0, len(names)))]
            if (side == "L" and c == only_right) or (side == "R" and c == only_left):
                continue
            s = int(rng.integers(0, lens[c] - 400))
            e = s + int(rng.integers(0, 400))
            strand = "INDEPENDENT" if rng.random() < 0.8 else "FORWARD"
            out.append((st.ReferenceRegion(c, s, e, strand), f"{side}{i}"))
        return out
    L, R = rdd(600, "L"), rdd(500, "R")
    Lu = [(st.ReferenceRegion(r.referenceName, r.start, r.end), v) for r, v in L]
    Ru = [(st.ReferenceRegion(r.referenceName, r.start, r.end), v) for r, v in R]
    bounds = {n: st.ReferenceRegion(n, 0, lens[n]) for n in names}
    ops = [lambda: st.DistributedIntersection(L, R, ctx=ctx).compute(),
           lambda: st.DistributedWindow(L, R, threshold=300, ctx=ctx).compute(),
           lambda: st.DistributedSubtract(L, R, ctx=ctx).compute(),
           lambda: st.DistributedMerge(L, ctx=ctx).compute(),
           lambda: st.UnstrandedCluster(L, ctx=ctx).compute(),
           lambda: st.StrandedCluster(L, ctx=ctx).compute(),
           lambda: st.SingleClosest(Lu, Ru, ctx=ctx).compute(),
           lambda: st.SingleClosestSingleOverlap(Lu, Ru, ctx=ctx).compute(),
           lambda: st.DistributedComplement(L, referenceNameBounds=bounds, ctx=ctx).compute()]
    one = [op() for op in ops]
    assert len(st._space_for([r for r, _ in L], [r for r, _ in R]).spaces) == 1
    monkeypatch.setattr(st, "SPAN_CAP", 26000)
    assert len(st._space_for([r for r, _ in L], [r for r, _ in R]).spaces) >= 3
    cut = [op() for op in ops]
    for k, (x, y) in enumerate(zip(one, cut)):
        assert x == y, k
    assert all(len(x) for x in one)
    with pytest.raises(LimeError):
        monkeypatch.setattr(st, "SPAN_CAP", 1000)  # every contig is longer
        ops[0]()


def _sub_equal(res, exp):
    og, oe = np.argsort(res["a_row"], kind="stable"), np.argsort(exp["a_row"], kind="stable")
    for key in ("contig", "start", "end", "a_row", "b_row"):
        assert list(res[key][og]) == list(exp[key][oe]), key


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("t", [0, -3])
def test_subtract_runs_path(ctx, mode, t):
    # threshold <= 0 takes the runs path (a block = one of B's merge runs cut
    # at the left row's end): dense ties, zero-width rows (zero-width heads
    # duplicate their block), duplicates and book-ended rows on short
    # contigs, then deep coverage (C2-like: ~300 hits per left row)
    for seed in range(40):
        rng = np.random.default_rng(1000 + seed)
        A, B = random_sets(rng, 300, 300, n_contigs=2, contig_len=400, max_len=30,
                           zero_frac=0.2, dup_frac=0.2, book_frac=0.3)
        sp = space_for(2, 400)
        res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t,
                           mode).to_host()
        _sub_equal(res, oracle.subtract(A, B, t, mode))
    rng = np.random.default_rng(77)
    A, B = random_sets(rng, 20000, 20000, n_contigs=2, contig_len=100000, max_len=3000,
                       zero_frac=0.02, dup_frac=0.02, book_frac=0.05)
    sp = space_for(2, 100000)
    res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t, mode).to_host()
    _sub_equal(res, oracle.subtract(A, B, t, mode))


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("t", [0, -3])
def test_subtract_local_scan(ctx, mode, t, monkeypatch):
    # B without zero-width rows and every 1024-row tile's window within 1536
    # of B's rows takes k_sub_fused<true>: the window's prefix max and run ids
    # by two block scans, no merge scan of B.  Book-ended rows (run breaks),
    # duplicates, a 30-row same-start group (tie index), left rows before B
    # and past its end, B from a tenth to 1.4x A's density and rows up to
    # 4000 long; each against the oracle and the merge-scan path
    # (LIME_SUB_NO_LS), which must agree record for record
    for seed, na, nb, max_len in [(1, 9000, 900, 400), (2, 9000, 9000, 40),
                                  (3, 9000, 12600, 60), (4, 3000, 2000, 4000),
                                  (5, 20000, 15000, 200)]:
        rng = np.random.default_rng(5100 + seed)
        L = 60 * na
        A, B = random_sets(rng, na, nb, n_contigs=3, contig_len=L, max_len=max_len,
                           dup_frac=0.05, book_frac=0.2)
        keep = B[2] > B[1]  # (no zero-width rows in B)
        B = [x[keep] for x in B]
        B[0][:30], B[1][:30] = B[0][40], B[1][40]
        B[2][:30] = B[1][40] + rng.integers(1, 30, 30)
        A[1][:5], A[2][:5] = 0, 3  # before B
        A[0][5:10], A[1][5:10], A[2][5:10] = 2, L - 5, L  # past B's end
        sp = space_for(3, L)
        exp = oracle.subtract(A, B, t, mode)
        res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t,
                           mode).to_host()
        _sub_equal(res, exp)
        monkeypatch.setenv("LIME_SUB_NO_LS", "1")
        ref = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t,
                           mode).to_host()
        monkeypatch.delenv("LIME_SUB_NO_LS")
        _sub_equal(ref, exp)


@pytest.mark.gpu
def test_subtract_total_disagreement_fails(ctx, monkeypatch):
    # the fused subtract reruns at the first pass's exact total when its guess
    # overflows; a second pass that reports more than that must fail loudly
    # (LIME_TEST_SUB_SKEW=1 makes both passes report one past their capacity)
    # rather than return a result whose arrays were freed; the same call then
    # succeeds without the hook
    rng = np.random.default_rng(5200)
    A, B = random_sets(rng, 4000, 3000, n_contigs=2, contig_len=240000, max_len=300)
    keep = B[2] > B[1]
    B = [x[keep] for x in B]
    sp = space_for(2, 240000)
    a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
    monkeypatch.setenv("LIME_TEST_SUB_SKEW", "1")
    with pytest.raises(Exception, match="record total changed"):
        ctx.subtract(a, b, 0, SUBTRACT_LIME)
    monkeypatch.delenv("LIME_TEST_SUB_SKEW")
    _sub_equal(ctx.subtract(a, b, 0, SUBTRACT_LIME).to_host(),
               oracle.subtract(A, B, 0, SUBTRACT_LIME))


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("deep", [False, True])
def test_subtract_one_pass_and_two_pass(ctx, mode, deep):
    # threshold 0 over B's runs takes one of two launches: the one-pass
    # k_sub_fused (count, look-back placement, write) when B merges into at
    # least 1/64 as many runs as A has rows, else the count pass + a
    # write pass over the tiles with records (B covering A deeply).  The same
    # left rows against a sparse B (one pass) and that B plus long rows
    # covering nearly everything (two passes), with zero-width rows,
    # duplicates, book-ended rows and a 30-row same-start group (tie index)
    rng = np.random.default_rng(4242)
    L = 200_000
    A = random_sets(rng, 8000, 1, n_contigs=2, contig_len=L, max_len=400, zero_frac=0.05,
                    dup_frac=0.05, book_frac=0.1)[0]
    B = random_sets(rng, 4000, 1, n_contigs=2, contig_len=L, max_len=100, zero_frac=0.05,
                    dup_frac=0.05, book_frac=0.1)[0]
    B = [x.copy() for x in B]
    B[0][:30], B[1][:30] = B[0][40], B[1][40]
    B[2][:30] = B[1][40] + rng.integers(1, 300, 30)
    if deep:
        k = 300
        c = rng.integers(0, 2, k).astype(B[0].dtype)
        st = rng.integers(0, L - 30_000, k)
        B = [np.concatenate([B[0], c]), np.concatenate([B[1], st]),
             np.concatenate([B[2], st + rng.integers(5_000, 30_000, k)])]
    sp = space_for(2, L)
    sb = ctx.set_from_host(sp, *B)
    runs = ctx.merge(sb).n
    assert (runs * 64 >= len(A[0])) == (not deep)  # the launch this case is for
    res = ctx.subtract(ctx.set_from_host(sp, *A), sb, 0, mode).to_host()
    _sub_equal(res, oracle.subtract(A, B, 0, mode))


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
def test_subtract_sweeping_write_pass(ctx, mode, monkeypatch):
    # records under one per 16 blocks of 256 left rows (B covering A, C2's
    # shape) take the sweeping write pass (k_subtract<true, true, true>):
    # each workgroup tests 256 blocks and folds only those with records.
    # 120k left rows inside B's rows but for two narrow gaps between them,
    # a few rows past B and one crossing B's end: a handful of records in
    # both workgroups' sweeps
    rng = np.random.default_rng(77)
    L = 2_000_000
    n = 120_000
    st = np.sort(rng.integers(10, 1_400_000, n)).astype(np.uint32)
    A = [np.zeros(n, np.int32), st, st + rng.integers(1, 40, n).astype(np.uint32)]
    for i in (0, 255, 256, 30_000):  # left rows past B (their own records)
        A[1][i], A[2][i] = 1_900_000 + i, 1_900_010 + i
    A[1][-1], A[2][-1] = 1_499_990, 1_600_000  # crosses B's end
    o = np.lexsort((A[2], A[1], A[0]))
    A = [x[o] for x in A]
    B = [np.zeros(4, np.int32), np.array([0, 5, 500_001, 1_200_001], np.uint32),
         np.array([500_000, 400_000, 1_200_000, 1_500_000], np.uint32)]
    sp = space_for(1, L)
    # (B has no zero-width rows: without LIME_SUB_NO_LS this takes the local
    # scan's one pass)
    monkeypatch.setenv("LIME_SUB_NO_LS", "1")
    res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), 0, mode).to_host()
    exp = oracle.subtract(A, B, 0, mode)
    assert 0 < len(exp["start"]) * 16 < (n + 255) // 256
    assert len(set(exp["a_row"] // 65536)) == 2  # records in both sweeps
    _sub_equal(res, exp)

def test_bitset_and_past_sixteen_sets(ctx):
    # the fused AND paints 16 sets per kernel and chains the groups
    # (lime_bitset_and_from_device); lime_bitset_and_runs chains its words
    # past 16 bitsets.  16 and 17 sets: fused == chained words == sharded run
    # == the oracle's fold of intersect over the merged operands (A.4)
    from lime_amd.sharded import ShardedBitset
    from tests.test_gpu_configs import coalesce
    rng = np.random.default_rng(95)
    sp = space_for(2, 200000)
    # ~1500 rows of <= 2 kb per set: each covers ~97% of the bases, so the
    # AND of 17 keeps about two thirds in many runs
    sets = [random_sets(rng, 1500, 1, n_contigs=2, contig_len=200000, max_len=2000)[0]
            for _ in range(17)]
    dev = [_dev_rows(A) for A in sets]
    rows = [(len(A[0]), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr())
            for A, t in zip(sets, dev)]
    bits = [ctx.bitset_from_device(sp, *r) for r in rows]
    cur = oracle.merge(sets[0])
    for k in range(2, 18):
        m = oracle.merge(sets[k - 1])
        ix = oracle.intersect((cur["contig"], cur["start"], cur["end"]),
                              (m["contig"], m["start"], m["end"]))
        order = np.lexsort((ix["start"], ix["contig"]))
        cur = {key: np.asarray(ix[key])[order] for key in ("contig", "start", "end")}
        if k < 16:
            continue
        fused = ctx.bitset_and_from_device(sp, rows[:k])
        got = ctx.bitset_runs(0, fused).to_host()
        words = ctx.bitset_and(bits[:k]).to_host()
        assert len(got["start"]) > 100
        for key in ("contig", "start", "end"):
            assert got[key].tolist() == words[key].tolist()
        x = coalesce(cur["contig"], cur["start"], cur["end"])
        for a_, b_ in zip((got["contig"], got["start"], got["end"]), x):
            assert np.asarray(a_).tolist() == np.asarray(b_).tolist()
        out = ShardedBitset(ctx, sp).run(rows[:k], gather=True)
        gs = sp.offsets[np.asarray(got["contig"])] + np.asarray(got["start"], np.int64)
        assert out["runs"].numpy()[:, 0].tolist() == gs.tolist()
        out["result"].close()


def test_spaces_cached_per_context(ctx):
    # the context keeps one device copy of each space's offsets (keyed by the
    # offsets): sets and bitsets of different spaces, built and queried in
    # interleaved order, and a space destroyed and rebuilt, all stay exact
    rng = np.random.default_rng(97)
    lens_a = [50000, 50000, 50000, 777]
    lens_b = [60000, 40000, 50000]
    A, _ = random_sets(rng, 3000, 1, n_contigs=3, contig_len=40000, max_len=400)
    B, _ = random_sets(rng, 3000, 1, n_contigs=3, contig_len=40000, max_len=400)
    for rep in range(2):
        spa, spb = Space(NAMES[:4], lens_a), Space(NAMES[:3], lens_b)
        sa, sb = ctx.set_from_host(spa, *A), ctx.set_from_host(spb, *B)
        ca = ctx.complement(spa, sa).to_host()
        cb = ctx.complement(spb, sb).to_host()
        ea, eb = oracle.complement(A, lens_a), oracle.complement(B, lens_b)
        for k in ("contig", "start", "end"):
            assert list(ca[k]) == list(ea[k]), (rep, k)
            assert list(cb[k]) == list(eb[k]), (rep, k)
        # the bit-per-base NOT over each space: the same gaps, book-ended
        # zero-width gaps aside (Appendix A.4)
        da, db = _dev_rows(A), _dev_rows(B)
        na = ctx.bitset_runs(1, ctx.bitset_from_device(spa, len(A[0]),
                                                       *(x.data_ptr() for x in da))).to_host()
        nb = ctx.bitset_runs(1, ctx.bitset_from_device(spb, len(B[0]),
                                                       *(x.data_ptr() for x in db))).to_host()
        assert sum(e - s for s, e in zip(na["start"], na["end"])) == \
            sum(e - s for s, e in zip(ea["start"], ea["end"]))
        assert sum(e - s for s, e in zip(nb["start"], nb["end"])) == \
            sum(e - s for s, e in zip(eb["start"], eb["end"]))
        del sa, sb, spa, spb


def test_bitset_runs_dense_tile_falls_back(ctx):
    # a tile with more events than the extraction's per-tile stage (2048):
    # 3000 one-base runs two bases apart in the first 131072-base tile, plus
    # a sparse tail; the runs come back exact either way
    rng = np.random.default_rng(5)
    dense = np.arange(3000, dtype=np.int64) * 2
    tail = np.sort(rng.choice(np.arange(300000, 990000, 7), 500, replace=False)).astype(np.int64)
    starts = np.concatenate([dense, tail])
    ends = starts + 1
    contig = np.zeros(len(starts), np.int32)
    sp = Space(NAMES[:1], [1_000_000])
    dev = _dev_rows((contig, starts, ends))
    bs = ctx.bitset_from_device(sp, len(starts), *(x.data_ptr() for x in dev))
    got = ctx.bitset_runs(0, bs).to_host()
    assert got["start"].tolist() == starts.tolist()
    assert got["end"].tolist() == ends.tolist()


@pytest.mark.parametrize("mode", [SUBTRACT_LIME, SUBTRACT_SET])
@pytest.mark.parametrize("t", [0, 1])
def test_subtract_many_same_start_rows(ctx, mode, t):
    # PCR-duplicate-like B: thousands of rows sharing a start, mostly
    # identical, some with other ends (in random input order, so the head --
    # the min (end, row) among the same-start hits, Subtract.scala:103-108 --
    # is not the first of them), zero-width ones, and groups spanning and
    # inside the left rows.  Past TIE_G such rows the head comes from the tie
    # index (one search), not a walk per left row (the O(n_A x D) cliff).
    rng = np.random.default_rng(2024 + t)
    L = 200_000
    a_s = rng.integers(0, L - 3000, 8000)
    A = (np.zeros(8000, np.int32), a_s, a_s + rng.integers(1, 3000, 8000))
    parts = []
    for start, d in ((1000, 12000), (50_000, 3000), (120_000, 40), (150_000, 17)):
        e = np.full(d, start + 5000)
        k = rng.random(d)
        e[k < 0.03] = start + 2000
        e[(k >= 0.03) & (k < 0.05)] = start  # zero-width
        parts.append((np.full(d, start), e))
    bs_ = rng.integers(0, L - 3000, 4000)
    parts.append((bs_, bs_ + rng.integers(0, 3000, 4000)))
    s = np.concatenate([p[0] for p in parts])
    e = np.concatenate([p[1] for p in parts])
    perm = rng.permutation(len(s))
    B = (np.zeros(len(s), np.int32), s[perm], e[perm])
    sp = space_for(1, L)
    res = ctx.subtract(ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B), t, mode).to_host()
    _sub_equal(res, oracle.subtract(A, B, t, mode))
