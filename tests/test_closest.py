"""closest: SingleClosest, Closest.scala:34-214.

CPU: the oracle's restatement (lo_closest) against ClosestSuite's arrays and an
independent pure-Python transcription of the sweep; and the engine's parallel
decomposition of that sweep (right pointer = prefix max of per-left stops until
the first active "jag", cache head = fixed point of a monotone map), restated
here in Python, against the oracle on thousands of random cases.
GPU: the engine through the C-ABI against the oracle, record for record."""
import bisect
import os
import random

import numpy as np
import pytest

from oracle import oracle
from tests.util import GOLDEN, expected, random_sets, ranked, read_bed_py

NONE = None


def load(name, rank):
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, name))
    return np.array([rank[c] for c in chrom], np.int32), s, e


def suite_pairs(mode):
    a, _, _, _ = read_bed_py(os.path.join(GOLDEN, "intersect_with_overlap_00.bed"))
    b, _, _, _ = read_bed_py(os.path.join(GOLDEN, "intersect_with_overlap_01.bed"))
    rank = ranked(a + b)
    names = sorted(rank, key=rank.get)
    A = load("intersect_with_overlap_00.bed", rank)
    B = load("intersect_with_overlap_01.bed", rank)
    got = oracle.closest(A, B, mode)
    return [[[names[c], int(s), int(e)], [names[B[0][r]], int(B[1][r]), int(B[2][r])]]
            for c, s, e, r in zip(got["contig"], got["start"], got["end"], got["b_row"])]


def test_oracle_suite_single_closest():
    # ClosestSuite.scala:8-49: all 24 bedtools-derived pairs, in order
    assert suite_pairs(oracle.CLOSEST) == [list(map(list, p)) for p in expected()["closest"]]


def test_oracle_suite_single_overlap():
    # ClosestSuite.scala:51-89 (SingleClosestSingleOverlap): all 21 pairs
    assert suite_pairs(oracle.CLOSEST_SINGLE) == \
        [list(map(list, p)) for p in expected()["closest_single_overlap"]]


# ---------------------------------------------------------------- helpers
def _covers(a, b):
    return a[0] == b[0] and a[2] > b[1] and a[1] < b[2]


def _dist(a, b):
    if a[0] != b[0]:
        return NONE
    if _covers(a, b):
        return 0
    return b[1] - a[2] + 1 if b[1] >= a[2] else a[1] - b[2] + 1


_SORD = {0: 2, 1: 0, 2: 1, 3: 3}


def _sorted_rows(X, st):
    c, s, e = X
    rows = [(int(c[i]), int(s[i]), int(e[i]), i, int(st[i])) for i in range(len(s))]
    return sorted(rows, key=lambda r: (r[0], r[1], r[2], _SORD[r[4]], r[3]))


def sweep_py(L, R):
    """Closest.scala:160-213 over SetTheory.scala:131-187, transcribed
    directly (currentClosest starts on no contig)."""
    C = (-1, 0, 0)
    cache, j, out = [], 0, []
    big = 2 ** 63 - 1
    for l in L:
        while j < len(R):
            c = R[j]
            if c[0] != l[0]:
                break
            if l[0] != C[0] or _dist(l, c) <= (big if _dist(l, C) is None else _dist(l, C)):
                C = c
                cache.append(c)
                j += 1
            else:
                break
        dC = _dist(l, C)
        idx = next((k for k, c in enumerate(cache)
                    if not (c[0] != l[0] or _dist(l, c) > (0 if dC is None else dC))), -1)
        if idx > 0:
            cache = cache[idx:]
        tgt = big if dC is None else dC
        out += [(l[3], c[3]) for c in cache if _dist(l, c) == tgt]
    return out


def decomposed_py(L, R, n_contigs):
    """The engine's decomposition (lime_amd/csrc/closest.hip), step by step."""
    nR, nL = len(R), len(L)
    starts = [r[1] for r in R]
    ends = [r[2] for r in R]
    rb = [bisect.bisect_left([(r[0]) for r in R], c) for c in range(n_contigs + 1)]
    jag = [k > rb[R[k][0]] and ends[k - 1] > ends[k] for k in range(nR)]   # k_jags
    A, N = [], []                                                         # k_stops
    for l in L:
        lo, hi = rb[l[0]], rb[l[0] + 1]
        a = bisect.bisect_left(starts, l[2], lo, hi)
        if a == hi:
            n = hi
        elif a > lo and _dist(l, R[a - 1]) < _dist(l, R[a]):
            n = a
        else:
            n = bisect.bisect_right(starts, starts[a], a, hi)
        A.append(a)
        N.append(n)
    U = list(np.maximum.accumulate(N)) if nL else []                      # prefix max
    stuck = {}                                                            # k_stuck
    for i, l in enumerate(L):
        lo = max(U[i - 1] if i else 0, rb[l[0]] + 1)
        k = next((k for k in range(lo, A[i]) if jag[k] and ends[k] <= l[1]), None)
        if k is not None and l[0] not in stuck:
            stuck[l[0]] = (i, k)

    def ptr(i):
        c = L[i][0]
        return stuck[c][1] if c in stuck and i >= stuck[c][0] else U[i]
    live, alive, first = {}, True, True                                   # liveness
    lcs = sorted(set(l[0] for l in L))
    for x, c in enumerate(lcs):
        if first:
            alive, first = rb[c] == 0, False
        live[c] = alive
        if alive:
            last = max(i for i, l in enumerate(L) if l[0] == c)
            alive = ptr(last) == rb[c + 1]
            if alive and x + 1 < len(lcs):
                alive = rb[c + 1] == rb[lcs[x + 1]]
    pmax = list(np.maximum.accumulate(ends)) if nR else []
    J, D, P = [], [], []                                                  # k_fresh

    def near_from(i, x, fresh):
        l, d, a, j = L[i], D[i], A[i], J[i]
        T = l[1] + 1 - d
        hi = min(a, j)
        if x < hi:
            if fresh:
                k = bisect.bisect_left(pmax, T, x, hi)
            else:
                k = next((k for k in range(x, hi) if ends[k] >= T), hi)
            if k < hi:
                return k
        k = max(x, a)
        return k if k < j and starts[k] <= l[2] + d - 1 else x
    for i, l in enumerate(L):
        j = ptr(i)
        J.append(j)
        r0 = rb[l[0]]
        if not live[l[0]] or j <= r0:
            D.append(NONE)
            P.append(r0)
            continue
        D.append(_dist(l, R[j - 1]))
        P.append(near_from(i, r0, True))
    p = list(np.maximum.accumulate(P)) if nL else []                      # prefix max
    rounds = 0
    while True:                                                           # k_prune_round
        rounds += 1
        q = [p[i] if D[i] is NONE else
             max(p[i], near_from(i, max(p[i - 1] if i else 0, rb[L[i][0]]), False))
             for i in range(nL)]
        if q == p:
            break
        p = q
    out = []                                                              # k_emit
    for i, l in enumerate(L):
        if D[i] is not NONE:
            out += [(l[3], R[k][3]) for k in range(p[i], J[i]) if _dist(l, R[k]) == D[i]]
    return out, rounds


def _case(seed):
    rng = random.Random(seed)
    nc = rng.choice([1, 1, 2, 3, 4])
    span = rng.choice([60, 300, 3000])
    ml = rng.choice([2, 20, 200, 2000])

    def gen(n):
        c = np.array([rng.randrange(nc) for _ in range(n)], np.int32)
        s = np.array([rng.randrange(span) for _ in range(n)], np.int64)
        ln = np.array([0 if rng.random() < 0.1 else rng.randrange(1, ml + 1) for _ in range(n)],
                      np.int64)
        st = np.array([rng.randrange(4) for _ in range(n)], np.int8)
        return (c, s, s + ln), st
    (A, sa), (B, sb) = gen(rng.randrange(0, 50)), gen(rng.randrange(0, 50))
    return nc, A, sa, B, sb


@pytest.mark.parametrize("block", range(4))
def test_oracle_vs_transcribed_sweep(block):
    for seed in range(block * 400, block * 400 + 400):
        nc, A, sa, B, sb = _case(seed)
        exp = oracle.closest((*A, sa), (*B, sb))
        got = sweep_py(_sorted_rows(A, sa), _sorted_rows(B, sb))
        assert got == list(zip(exp["a_row"].tolist(), exp["b_row"].tolist())), seed


@pytest.mark.parametrize("block", range(4))
def test_decomposition_vs_oracle(block):
    worst = 0
    for seed in range(block * 400, block * 400 + 400):
        nc, A, sa, B, sb = _case(seed)
        exp = oracle.closest((*A, sa), (*B, sb))
        got, rounds = decomposed_py(_sorted_rows(A, sa), _sorted_rows(B, sb), nc)
        assert got == list(zip(exp["a_row"].tolist(), exp["b_row"].tolist())), seed
        worst = max(worst, rounds)
    assert worst < 16  # rounds to the fixed point (incl. the confirming one): 1-7 here


# -------------------------------------------------------------------- GPU
def _space(nc, ln):
    from lime_amd import Space
    return Space([f"chr{i + 1}" for i in range(nc)], [ln] * nc)


def _gpu_vs_oracle(ctx, sp, A, sa, B, sb, mode=0):
    a = ctx.set_from_host_stranded(sp, *A, sa)
    b = ctx.set_from_host_stranded(sp, *B, sb)
    plan = ctx.closest(a, b, mode)
    exp = oracle.closest((*A, sa), (*B, sb), mode)
    assert plan.n == len(exp["start"])
    p = plan.fill_host()
    assert p["a_row"].tolist() == exp["a_row"].tolist()
    assert p["b_row"].tolist() == exp["b_row"].tolist()
    assert p["start"].tolist() == exp["start"].tolist()
    assert p["end"].tolist() == exp["end"].tolist()
    assert plan.checksum() == oracle.checksum_pairs(exp)
    return plan.n


@pytest.mark.gpu
def test_gpu_suite(ctx):
    from lime_amd.set_theory import ReferenceRegion, SingleClosest

    def keyed(name):
        chrom, s, e, nm = read_bed_py(os.path.join(GOLDEN, name))
        return [(ReferenceRegion.unstranded(c, x, y), (c, x, y)) for c, x, y in zip(chrom, s, e)]
    out = SingleClosest(keyed("intersect_with_overlap_00.bed"),
                        keyed("intersect_with_overlap_01.bed"), None, ctx=ctx).compute()
    got = [[[r.referenceName, r.start, r.end], [v[1][0], int(v[1][1]), int(v[1][2])]]
           for r, v in out]
    assert got == [list(map(list, p)) for p in expected()["closest"]]


@pytest.mark.gpu
def test_gpu_random_small(ctx):
    for seed in range(300):
        nc, A, sa, B, sb = _case(seed)
        _gpu_vs_oracle(ctx, _space(nc, 6000), A, sa, B, sb)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,max_len,zero,dup", [
    (1, 20000, 300, 0.0, 0.0), (2, 20000, 3000, 0.1, 0.05), (3, 50000, 40, 0.05, 0.2),
    (4, 200000, 5000, 0.02, 0.02)])
def test_gpu_random_large(ctx, seed, n, max_len, zero, dup):
    rng = np.random.default_rng(seed)
    A, B = random_sets(rng, n, n, n_contigs=3, contig_len=40 * n, max_len=max_len,
                       zero_frac=zero, dup_frac=dup, book_frac=0.05)
    sa = rng.integers(0, 4, n).astype(np.int8)
    sb = rng.integers(0, 4, n).astype(np.int8)
    assert _gpu_vs_oracle(ctx, _space(3, 40 * n), A, sa, B, sb) > 0


@pytest.mark.gpu
def test_gpu_live_contigs(ctx):
    # every contig of the left side keeps a live sweep: rights cover each
    # left contig to its end, so the pointer crosses contigs
    rng = np.random.default_rng(9)
    n = 30000
    c = np.sort(rng.integers(0, 4, n)).astype(np.int32)
    s = rng.integers(0, 99900, n).astype(np.int64)
    A = (c, s, s + rng.integers(1, 50, n))
    cb = np.repeat(np.arange(4, dtype=np.int32), 2)
    B = (cb, np.tile(np.array([0, 99990], np.int64), 4), np.tile(np.array([5, 100000]), 4))
    z = lambda k: np.zeros(k, np.int8)
    assert _gpu_vs_oracle(ctx, _space(4, 100000), A, z(n), B, z(8)) >= n


@pytest.mark.gpu
def test_gpu_empty_and_errors(ctx):
    from lime_amd import LimeError
    sp = _space(2, 1000)
    e = (np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, np.int64))
    one = (np.zeros(1, np.int32), np.array([5], np.int64), np.array([9], np.int64))
    z = lambda k: np.zeros(k, np.int8)
    assert _gpu_vs_oracle(ctx, sp, e, z(0), one, z(1)) == 0
    assert _gpu_vs_oracle(ctx, sp, one, z(1), e, z(0)) == 0
    a = ctx.set_from_host(sp, *one)
    b = ctx.set_from_host_stranded(sp, *one, z(1))
    with pytest.raises(LimeError):
        ctx.closest(a, b)


@pytest.mark.gpu
def test_gpu_device_stranded_sets(ctx):
    # sets built from device rows (lime_set_create_device_stranded, no strand
    # codes) give the same closest records as host-built stranded sets
    import torch
    rng = np.random.default_rng(21)
    n = 40000
    A, B = random_sets(rng, n, n, n_contigs=2, contig_len=400000, max_len=2000, zero_frac=0.05,
                       dup_frac=0.05, book_frac=0.05)
    sp = _space(2, 400000)

    def dev_set(X):
        t = [torch.tensor(np.asarray(x, np.int32), device="cuda") for x in X]
        s = ctx.set_from_device_stranded(sp, len(X[1]), *[x.data_ptr() for x in t])
        torch.cuda.synchronize()
        return s, t
    (a, ta), (b, tb) = dev_set(A), dev_set(B)
    z = np.zeros(n, np.int8)
    exp = oracle.closest((*A, z), (*B, z))
    plan = ctx.closest(a, b)
    p = plan.fill_host()
    assert p["a_row"].tolist() == exp["a_row"].tolist()
    assert p["b_row"].tolist() == exp["b_row"].tolist()


@pytest.mark.gpu
def test_gpu_c2_density(ctx):
    # C2's density (depth ~82, len U[50,5000]) on hg38/100 with 2 x 1e6 rows:
    # count and order-free checksum of ~2.5e7 records == oracle
    from lime_amd import Space, synth
    lens = np.array(list(synth.HG38.values())) // 100
    sp = Space(list(synth.HG38.keys()), lens.tolist())
    A = synth.uniform(lens, 1_000_000, 0xA, 50, 5000)
    B = synth.uniform(lens, 1_000_000, 0xB, 50, 5000)
    # synth indexes contigs in HG38 order; the space numbers them in Java
    # String order, which both sides must share (it orders the sweep)
    m = np.array([sp.index[nm] for nm in synth.HG38], np.int32)
    A = (m[A[0]], np.asarray(A[1], np.int64), np.asarray(A[2], np.int64))
    B = (m[B[0]], np.asarray(B[1], np.int64), np.asarray(B[2], np.int64))
    z = np.zeros(1_000_000, np.int8)
    a = ctx.set_from_host_stranded(sp, *A, z)
    b = ctx.set_from_host_stranded(sp, *B, z)
    plan = ctx.closest(a, b)
    exp = oracle.closest((*A, z), (*B, z))
    assert plan.n == len(exp["start"]) > 1_000_000
    assert plan.checksum() == oracle.checksum_pairs(exp)


# ------------------------------------------- SingleClosestSingleOverlap (mode 1)
@pytest.mark.gpu
def test_gpu_suite_single_overlap(ctx):
    from lime_amd.set_theory import ReferenceRegion, SingleClosestSingleOverlap

    def keyed(name):
        chrom, s, e, nm = read_bed_py(os.path.join(GOLDEN, name))
        return [(ReferenceRegion.unstranded(c, x, y), (c, x, y)) for c, x, y in zip(chrom, s, e)]
    out = SingleClosestSingleOverlap(keyed("intersect_with_overlap_00.bed"),
                                     keyed("intersect_with_overlap_01.bed"), None,
                                     ctx=ctx).compute()
    got = [[[r.referenceName, r.start, r.end], [v[1][0], int(v[1][1]), int(v[1][2])]]
           for r, v in out]
    assert got == [list(map(list, p)) for p in expected()["closest_single_overlap"]]


@pytest.mark.gpu
def test_gpu_single_overlap_random(ctx):
    for seed in range(300):
        nc, A, sa, B, sb = _case(seed)
        _gpu_vs_oracle(ctx, _space(nc, 6000), A, sa, B, sb, mode=1)
    for seed, n, ml in [(5, 20000, 300), (6, 20000, 3000), (7, 100000, 5000)]:
        rng = np.random.default_rng(seed)
        A, B = random_sets(rng, n, n, n_contigs=3, contig_len=40 * n, max_len=ml,
                           zero_frac=0.05, dup_frac=0.05, book_frac=0.05)
        sa = rng.integers(0, 4, n).astype(np.int8)
        sb = rng.integers(0, 4, n).astype(np.int8)
        assert _gpu_vs_oracle(ctx, _space(3, 40 * n), A, sa, B, sb, mode=1) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["0", "1"])
def test_gpu_sequential_fixed_point(ctx, monkeypatch, cap):
    # past the Jacobi round cap the in-order per-contig recursion finishes the
    # cache-head chain (an adversarial chain needs O(n) rounds);
    # forcing it from round 0 or 1 must give the oracle's answer
    monkeypatch.setenv("LIME_CLOSEST_MAX_ROUNDS", cap)
    seq = 0
    for seed in range(60):
        nc, A, sa, B, sb = _case(seed)
        sp = _space(nc, 6000)
        a = ctx.set_from_host_stranded(sp, *A, sa)
        b = ctx.set_from_host_stranded(sp, *B, sb)
        plan = ctx.closest(a, b, 0)
        rounds, used = plan.closest_rounds()
        assert rounds <= int(cap)
        seq += used
        _gpu_vs_oracle(ctx, sp, A, sa, B, sb)
    rng = np.random.default_rng(5)
    n = 100000
    A, B = random_sets(rng, n, n, n_contigs=3, contig_len=40 * n, max_len=3000,
                       zero_frac=0.05, dup_frac=0.05, book_frac=0.05)
    s_a = rng.integers(0, 4, n).astype(np.int8)
    s_b = rng.integers(0, 4, n).astype(np.int8)
    assert _gpu_vs_oracle(ctx, _space(3, 40 * n), A, s_a, B, s_b) > 0
    assert seq == 60 if cap == "0" else seq >= 0


@pytest.mark.gpu
def test_gpu_rounds_recorded(ctx):
    rng = np.random.default_rng(6)
    n = 50000
    A, B = random_sets(rng, n, n, n_contigs=3, contig_len=40 * n, max_len=3000)
    s_a = np.zeros(n, np.int8)
    sp = _space(3, 40 * n)
    plan = ctx.closest(ctx.set_from_host_stranded(sp, *A, s_a),
                       ctx.set_from_host_stranded(sp, *B, s_a), 0)
    rounds, used = plan.closest_rounds()
    assert 1 <= rounds <= 32 and not used
