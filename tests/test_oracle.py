"""Pin the CPU oracle (oracle/lime_oracle.c) before trusting it:
  1. against every golden vector the reference's hot-path suites hold
     (IntersectionSuite, SubtractSuite, MergeSuite, ComplementSuite), on the
     verbatim fixture files;
  2. against brute-force restatements of Appendix A on seeded inputs.
CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle
from tests.util import (GOLDEN, expected, java_key, random_sets, ranked, read_bed_py,
                        read_genome_py)


def load(name, rank):
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, name))
    return np.array([rank[c] for c in chrom], np.int32), s, e


def regions(res, names):
    return [[names[c], int(s), int(e)] for c, s, e in zip(res["contig"], res["start"],
                                                           res["end"])]


@pytest.fixture(scope="module")
def io():
    a, _, _, _ = read_bed_py(os.path.join(GOLDEN, "intersect_with_overlap_00.bed"))
    b, _, _, _ = read_bed_py(os.path.join(GOLDEN, "intersect_with_overlap_01.bed"))
    rank = ranked(a + b)
    names = sorted(rank, key=rank.get)
    return load("intersect_with_overlap_00.bed", rank), load("intersect_with_overlap_01.bed",
                                                             rank), names


def test_intersection_suite(io):
    # IntersectionSuite.scala:17-25 zips the output with 5 regions; the true
    # result has 7 (two exact-duplicate matches missing from the array, Q10).
    A, B, names = io
    got = regions(oracle.intersect(A, B), names)
    exp = expected()
    assert got[:5] == exp["intersection_prefix"]
    assert got == exp["intersection_full"]


def test_subtract_suite(io):
    # SubtractSuite.scala:20-39: exact 18 regions, in order
    A, B, names = io
    got = oracle.subtract(A, B)
    assert regions(got, names) == expected()["subtract"]
    # every left row that meets no right row comes back whole with None
    assert (got["b_row"] == -1).sum() == 17
    # lime and set modes agree whenever a left row meets <= 1 block
    assert regions(oracle.subtract(A, B, mode=oracle.SUB_SET), names) == expected()["subtract"]


def test_window_suite():
    # WindowSuite.scala:8-34: left intersect_with_overlap_00, right
    # window_with_overlap_01, default distance 1000; all 10 bedtools pairs
    a, _, _, _ = read_bed_py(os.path.join(GOLDEN, "intersect_with_overlap_00.bed"))
    b, _, _, _ = read_bed_py(os.path.join(GOLDEN, "window_with_overlap_01.bed"))
    rank = ranked(a + b)
    names = sorted(rank, key=rank.get)
    A = load("intersect_with_overlap_00.bed", rank)
    B = load("window_with_overlap_01.bed", rank)
    got = oracle.window(A, B, 1000)
    pairs = [[[names[c], int(s), int(e)],
              [names[B[0][r]], int(B[1][r]), int(B[2][r])]]
             for c, s, e, r in zip(got["contig"], got["start"], got["end"], got["b_row"])]
    assert pairs == expected()["window"]


def nearby_brute(a, b, d):
    """ADAM isNearby restated independently: same contig, overlap (strict,
    Appendix A) or gap + 1 <= d."""
    (ac, as_, ae), (bc, bs, be) = a, b
    out = []
    for i in range(len(as_)):
        for j in range(len(bs)):
            if ac[i] != bc[j]:
                continue
            if ae[i] > bs[j] and as_[i] < be[j]:
                dist = 0
            elif bs[j] >= ae[i]:
                dist = bs[j] - ae[i] + 1
            else:
                dist = as_[i] - be[j] + 1
            if dist <= d:
                out.append((int(i), int(j)))
    return sorted(out)


@pytest.mark.parametrize("seed,d", [(51, 1), (52, 7), (53, 150), (54, 1000)])
def test_window_vs_brute(seed, d):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 300, 250, n_contigs=3, contig_len=6000, max_len=200,
                       zero_frac=0.1, dup_frac=0.05, book_frac=0.1)
    got = oracle.window(A, B, d)
    assert sorted(zip(got["a_row"].tolist(), got["b_row"].tolist())) == nearby_brute(A, B, d)
    # records carry the left row's own region
    assert (got["start"] == A[1][got["a_row"]]).all() and (got["end"] == A[2][got["a_row"]]).all()


def test_cluster_suite():
    # ClusterSuite.scala:8-16: UnstrandedCluster of cpg_20merge.bed is one
    # cluster (the Merge fold, strand-blind, keyed by the first member)
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, "cpg_20merge.bed"))
    rank = ranked(chrom)
    res = oracle.merge((np.array([rank[c] for c in chrom], np.int32), s, e))
    assert len(res["start"]) == 1 and (res["run_of_row"] == 0).all()


@pytest.mark.parametrize("seed", [91, 92])
def test_stranded_merge_fold(seed):
    # lo_merge with strands = the SetTheory.scala:208-225 fold restated here
    # independently: RegionOrdering (name, start, end, bdg-formats Strand
    # ordinal FORWARD < REVERSE < INDEPENDENT < UNKNOWN), new run when the row
    # does not strictly overlap the head hull or has another strand
    rng = np.random.default_rng(seed)
    (c, s, e), _ = random_sets(rng, 1500, 1, n_contigs=2, contig_len=8000, max_len=300,
                               zero_frac=0.05, dup_frac=0.1, book_frac=0.05)
    st = rng.integers(0, 4, len(c)).astype(np.int8)
    ordv = {0: 2, 1: 0, 2: 1, 3: 3}
    order = sorted(range(len(c)), key=lambda i: (c[i], s[i], e[i], ordv[int(st[i])], i))
    runs, rid, hull = [], np.zeros(len(c), np.int64), None
    for i in order:
        if hull and c[i] == hull[0] and s[i] < hull[2] and e[i] > hull[1] and st[i] == hull[3]:
            hull = (hull[0], min(hull[1], s[i]), max(hull[2], e[i]), hull[3])
            runs[-1] = hull
        else:
            hull = (c[i], s[i], e[i], st[i])
            runs.append(hull)
        rid[i] = len(runs) - 1
    got = oracle.merge((c, s, e, st))
    assert list(zip(got["contig"].tolist(), got["start"].tolist(), got["end"].tolist())) == \
        [(int(a), int(b), int(x)) for a, b, x, _ in runs]
    assert got["run_of_row"].tolist() == rid.tolist()


def test_merge_suite():
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, "cpg_20merge.bed"))
    rank = ranked(chrom)
    res = oracle.merge((np.array([rank[c] for c in chrom], np.int32), s, e))
    assert len(res["start"]) == expected()["merge_count"]  # MergeSuite.scala:18
    assert (int(res["start"][0]), int(res["end"][0])) == (28735, 30000)
    assert (res["run_of_row"] == 0).all()


def test_complement_suite():
    gnames, glens = read_genome_py(os.path.join(GOLDEN, "genome.txt"))
    order = sorted(range(len(gnames)), key=lambda i: java_key(gnames[i]))
    names = [gnames[i] for i in order]
    lens = [glens[i] for i in order]
    rank = {n: i for i, n in enumerate(names)}
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, "cpg_20merge.bed"))
    res = oracle.complement((np.array([rank[c] for c in chrom], np.int32), s, e), lens)
    assert regions(res, names) == expected()["complement"]  # ComplementSuite.scala:19-114


def test_complement_unknown_contig():
    with pytest.raises(KeyError):
        oracle.complement((np.array([3], np.int32), np.array([0]), np.array([5])), [10, 10])


# ------------------------------------------------------------ brute force
def brute_pairs(A, B, t):
    out = []
    for i in range(len(A[0])):
        for j in range(len(B[0])):
            if A[0][i] != B[0][j]:
                continue
            a0, a1, b0, b1 = A[1][i], A[2][i], B[1][j], B[2][j]
            if not (a1 > b0 and a0 < b1):
                continue
            ov = min(a1, b1) - max(a0, b0)
            if ov >= t:
                out.append((int(A[0][i]), max(a0, b0), min(a1, b1), i, j))
    return sorted(out)


def tuples(res):
    return sorted(zip(res["contig"].tolist(), res["start"].tolist(), res["end"].tolist(),
                      res["a_row"].tolist(), res["b_row"].tolist()))


@pytest.mark.parametrize("seed,t,zero", [(1, 0, 0.0), (2, 0, 0.1), (3, 25, 0.0), (4, -3, 0.2),
                                         (5, 1, 0.1), (6, 120, 0.05)])
def test_intersect_vs_brute(seed, t, zero):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 300, 250, n_contigs=2, contig_len=6000, zero_frac=zero,
                       dup_frac=0.05, book_frac=0.1)
    assert tuples(oracle.intersect(A, B, t)) == brute_pairs(A, B, t)


def merge_components(A):
    """strict-overlap connected components (non-zero-width input)"""
    n = len(A[0])
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    for i in range(n):
        for j in range(i + 1, n):
            if A[0][i] == A[0][j] and A[2][i] > A[1][j] and A[1][i] < A[2][j]:
                parent[find(i)] = find(j)
    comp = {}
    for i in range(n):
        r = find(i)
        c, s, e = comp.get(r, (int(A[0][i]), 10**18, -1))
        comp[r] = (c, min(s, int(A[1][i])), max(e, int(A[2][i])))
    return sorted(comp.values())


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_merge_vs_components(seed):
    rng = np.random.default_rng(seed)
    A, _ = random_sets(rng, 400, 1, n_contigs=3, contig_len=8000, book_frac=0.2)
    res = oracle.merge(A)
    got = sorted(zip(res["contig"].tolist(), res["start"].tolist(), res["end"].tolist()))
    assert got == merge_components(A)


def base_sets(intervals):
    cov = {}
    for c, s, e in intervals:
        cov.setdefault(c, set()).update(range(s, e))
    return cov


def runs_of(bases):
    out = []
    for c in sorted(bases):
        xs = sorted(bases[c])
        i = 0
        while i < len(xs):
            j = i
            while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
                j += 1
            out.append((c, xs[i], xs[j] + 1))
            i = j + 1
    return out


@pytest.mark.parametrize("seed", [21, 22])
def test_complement_vs_bases(seed):
    rng = np.random.default_rng(seed)
    lens = [3000, 2500, 0, 4000]
    A, _ = random_sets(rng, 120, 1, n_contigs=2, contig_len=2500, max_len=200)
    cov = base_sets(zip(A[0].tolist(), A[1].tolist(), A[2].tolist()))
    comp = {c: set(range(lens[c])) - cov.get(c, set()) for c in range(len(lens))}
    res = oracle.complement(A, lens)
    got = sorted(zip(res["contig"].tolist(), res["start"].tolist(), res["end"].tolist()))
    assert got == runs_of(comp)


@pytest.mark.parametrize("seed,t", [(31, 0), (32, 10), (33, 1)])
def test_subtract_set_mode_vs_bases(seed, t):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 150, 150, n_contigs=2, contig_len=3000, max_len=250)
    res = oracle.subtract(A, B, t, mode=oracle.SUB_SET)
    got = {}
    for k in range(len(res["start"])):
        got.setdefault(int(res["a_row"][k]), []).append((int(res["start"][k]),
                                                          int(res["end"][k])))
    for i in range(len(A[0])):
        a0, a1 = int(A[1][i]), int(A[2][i])
        keep = set(range(a0, a1))
        for j in range(len(B[0])):
            if B[0][j] != A[0][i]:
                continue
            b0, b1 = int(B[1][j]), int(B[2][j])
            if a1 > b0 and a0 < b1 and min(a1, b1) - max(a0, b0) >= t:
                keep -= set(range(b0, b1))
        exp = [(c0, c1) for _, c0, c1 in runs_of({0: keep})]
        if keep == set(range(a0, a1)):
            exp = [(a0, a1)]
        assert got.get(i, []) == exp, i


def test_subtract_lime_multiblock_quirk():
    # Q5: a left row meeting two disjoint blocks gets remnants per block, in
    # reverse block order (Subtract.scala:103-114)
    A = (np.array([0], np.int32), np.array([0]), np.array([100]))
    B = (np.array([0, 0], np.int32), np.array([10, 50]), np.array([20, 60]))
    res = oracle.subtract(A, B)
    got = list(zip(res["start"].tolist(), res["end"].tolist(), res["b_row"].tolist()))
    assert got == [(0, 50, 1), (60, 100, 1), (0, 10, 0), (20, 100, 0)]
    res = oracle.subtract(A, B, mode=oracle.SUB_SET)
    assert list(zip(res["start"].tolist(), res["end"].tolist())) == [(0, 10), (20, 50),
                                                                      (60, 100)]


def test_zero_width_edges():
    # zero-width rows: merge keeps them apart from book-ended neighbours and
    # the zero-width subtract head is folded twice (duplicate block)
    A = (np.array([0, 0, 0], np.int32), np.array([5, 5, 7]), np.array([5, 10, 7]))
    res = oracle.merge(A)
    got = list(zip(res["start"].tolist(), res["end"].tolist()))
    assert got == [(5, 5), (5, 10)]
    L = (np.array([0], np.int32), np.array([0]), np.array([10]))
    R = (np.array([0], np.int32), np.array([4]), np.array([4]))
    res = oracle.subtract(L, R)
    assert list(zip(res["start"].tolist(), res["end"].tolist())) == [(0, 4), (4, 10), (0, 4),
                                                                      (4, 10)]
    # intersect: zero-width b strictly inside a hits (overlapsBy == 0 >= 0);
    # at a.start it does not (strict overlap)
    R2 = (np.array([0, 0], np.int32), np.array([0, 4]), np.array([0, 4]))
    res = oracle.intersect(L, R2)
    assert list(zip(res["start"].tolist(), res["end"].tolist(), res["b_row"].tolist())) == \
        [(4, 4, 1)]


# ------------------------------------------- contig-sharded drivers (MT)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mt_drivers_equal_single_partition(seed):
    # lo_intersect_mt / lo_merge_mt shard by contig over threads; every op is
    # contig-local, so they must reproduce the P = 1 restatement exactly
    # (records in order, checksums, run ids)
    from tests.util import random_sets
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 4000, 3000, n_contigs=5, contig_len=30000, max_len=400,
                       zero_frac=0.1, dup_frac=0.05, book_frac=0.1)
    for t in (0, 1, 30, -3):
        e = oracle.intersect(A, B, t)
        m = oracle.intersect_mt(5, A, B, t, records=True, nthreads=4)
        assert m["n"] == len(e["start"])
        for k in ("contig", "start", "end", "a_row", "b_row"):
            assert (m[k] == e[k]).all(), k
        assert (m["sum"], m["xor"]) == oracle.checksum_pairs(e)
        assert oracle.intersect_mt(5, A, B, t, nthreads=3)["sum"] == m["sum"]
    em = oracle.merge(A)
    mm = oracle.merge_mt(5, A, run_of_row=True, nthreads=4)
    for k in ("contig", "start", "end", "run_of_row"):
        assert (np.asarray(mm[k]) == np.asarray(em[k])).all(), k
    assert (mm["grp_sum"], mm["grp_xor"]) == oracle.grouping_checksum(em["run_of_row"])


@pytest.mark.parametrize("seed", [5, 6])
def test_mt_subtract_complement_equal_single_partition(seed):
    # lo_subtract_mt (both modes) / lo_complement_mt: the P = 1 restatement's
    # regions, by count and lime_result_checksum's region checksum
    from tests.util import random_sets
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, 4000, 3000, n_contigs=5, contig_len=30000, max_len=400,
                       zero_frac=0.1, dup_frac=0.05, book_frac=0.1)
    for t in (0, 1, 30, -3):
        for mode in (oracle.SUB_LIME, oracle.SUB_SET):
            e = oracle.subtract(A, B, t, mode)
            m = oracle.subtract_mt(5, A, B, t, mode, nthreads=4)
            assert m["n"] == len(e["start"])
            assert (m["sum"], m["xor"]) == oracle.result_checksum(e)
    genome = [30000, 31000, 32000, 33000, 34000, 40000]  # one contig without rows
    e = oracle.complement(A, genome)
    m = oracle.complement_mt(genome, A, nthreads=3)
    assert m["n"] == len(e["start"])
    assert (m["sum"], m["xor"]) == oracle.result_checksum(e)


def test_mt_drivers_on_reference_fixtures(golden):
    # the IntersectionSuite / MergeSuite inputs through the sharded drivers
    from tests.util import expected, ranked, read_bed_py
    a = read_bed_py(os.path.join(golden, "intersect_with_overlap_00.bed"))
    b = read_bed_py(os.path.join(golden, "intersect_with_overlap_01.bed"))
    rk = ranked(a[0] + b[0])
    A = (np.array([rk[c] for c in a[0]], np.int32), a[1], a[2])
    B = (np.array([rk[c] for c in b[0]], np.int32), b[1], b[2])
    m = oracle.intersect_mt(len(rk), A, B, records=True, nthreads=2)
    assert [[c, int(s), int(e)] for c, s, e in
            zip(["chr1"] * m["n"], m["start"], m["end"])] == expected()["intersection_full"]
    c = read_bed_py(os.path.join(golden, "cpg_20merge.bed"))
    mm = oracle.merge_mt(1, (np.zeros(len(c[1]), np.int32), c[1], c[2]))
    assert list(zip(mm["start"], mm["end"])) == [(28735, 30000)]
