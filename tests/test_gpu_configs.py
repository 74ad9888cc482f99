"""Parity at every BASELINE.json configuration (SURVEY.md 8(d) "Verification
at scale"), HIP engine through the C-ABI against the CPU oracle.

  C1  the CLI on C1's inputs: autosomal cpg.bed rows with i % 8 < 3 (i counts
      the autosomal rows in file order) and 10,000 uniform rows over the hg19
      autosomes of genome.txt (chr1-22 in file order, len U[200,2000], seed 1)
  C2  2 x 1e8 rows, uniform over hg38, len U[50,5000]: the pair count and the
      order-independent checksum of all ~1.63e10 pairs == the oracle's
      (contig-sharded, lo_intersect_mt), both as the fill computes it and
      over the records it stores in HBM; merge runs exact, grouping checksum
  C3  pile-up merge: exact runs + run_of_row at 1/50 scale; at full size
      (5e8 rows) exact runs and the checksum of every row's run
  C4  the hg38 bitset path (unsorted rows -> binned paint), A, B = 1e7 rows,
      len U[50,500]: NOT == oracle complement, AND-NOT == set-mode subtract of
      the merged runs, both after coalescing book-ended runs (Appendix A.4)
  C5  8-way AND at C5's density on hg38/8 (8 x 1.5625e7 rows, len U[10,40])
      == the oracle fold of intersect over the merged operands (A.4)

Inputs are made by the device generator (lime_synth_*), whose rows are pinned
bit-exact to the numpy restatement (test_device_synth_matches_numpy and the
prefix checks below); the oracle reads host copies of those same rows.
Integer work: every comparison is exact."""
import os
import subprocess

import numpy as np
import pytest

from lime_amd import Space, synth
from oracle import oracle
from tests.util import GOLDEN, read_bed_py, read_genome_py

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "lime-submit")


def hg38(scale=1):
    return Space(list(synth.HG38.keys()), [v // scale for v in synth.HG38.values()])


def device_rows(ctx, sp, n, seed, lo, hi, pile=None):
    """rows from the device generator: (torch tensors, host numpy copies)"""
    import torch
    c = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    e = torch.empty(n, dtype=torch.int32, device="cuda")
    if pile:
        ctx.synth_pileup(sp, n, seed, pile[0], pile[1], lo, hi, c.data_ptr(), s.data_ptr(),
                         e.data_ptr())
    else:
        ctx.synth_uniform(sp, n, seed, lo, hi, c.data_ptr(), s.data_ptr(), e.data_ptr())
    ctx.synchronize()
    host = (c.cpu().numpy(), s.cpu().numpy().view(np.uint32), e.cpu().numpy().view(np.uint32))
    # anchor: the first rows equal the numpy restatement of the generator
    k = min(n, 20000)
    ref = (synth.pileup(sp.lengths, k, seed, pile[0], pile[1], lo, hi) if pile
           else synth.uniform(sp.lengths, k, seed, lo, hi))
    for x, y in zip(host, ref):
        assert (x[:k].astype(np.int64) == y).all()
    return (c, s, e), host


def dset(ctx, sp, dev):
    c, s, e = dev
    return ctx.set_from_device(sp, c.numel(), c.data_ptr(), s.data_ptr(), e.data_ptr())


def dbits(ctx, sp, dev):
    c, s, e = dev
    return ctx.bitset_from_device(sp, c.numel(), c.data_ptr(), s.data_ptr(), e.data_ptr())


def region_checksum(contig, start, end, a_row=None, b_row=None):
    """numpy restatement of lime_result_checksum's region part"""
    from lime_amd.synth import mix64
    n = len(start)
    ff = np.full(n, 0xFFFFFFFF, np.uint64)
    a = ff if a_row is None else np.where(np.asarray(a_row) < 0, ff,
                                          np.asarray(a_row).astype(np.uint64))
    b = ff if b_row is None else np.where(np.asarray(b_row) < 0, ff,
                                          np.asarray(b_row).astype(np.uint64))
    s = np.asarray(start, np.uint64)
    e = np.asarray(end, np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(mix64(((s << np.uint64(32)) | e) ^ mix64((a << np.uint64(32)) | b)) +
                  np.asarray(contig, np.uint64))
        return int(np.sum(h, dtype=np.uint64)), int(np.bitwise_xor.reduce(h)) if n else 0


def coalesce(contig, start, end):
    """merge book-ended neighbours of sorted disjoint runs (Appendix A.4)"""
    c, s, e = (np.asarray(x, np.int64) for x in (contig, start, end))
    if len(s) == 0:
        return c, s, e
    join = np.zeros(len(s), bool)
    join[1:] = (c[1:] == c[:-1]) & (s[1:] == e[:-1])
    heads = np.flatnonzero(~join)
    tails = np.append(heads[1:] - 1, len(s) - 1)
    return c[heads], s[heads], e[tails]


def assert_runs_equal(got, exp):
    for x, y, k in zip(got, exp, ("contig", "start", "end")):
        x, y = np.asarray(x, np.int64), np.asarray(y, np.int64)
        assert len(x) == len(y), (k, len(x), len(y))
        bad = np.flatnonzero(x != y)
        assert len(bad) == 0, (k, int(bad[0]), int(x[bad[0]]), int(y[bad[0]]))


# ------------------------------------------------------------------ C1
def c1_inputs(tmp_path):
    chrom, s, e, name = read_bed_py(os.path.join(GOLDEN, "cpg.bed"))
    auto = {f"chr{i}" for i in range(1, 23)}
    rows = [i for i, c in enumerate(chrom) if c in auto]
    keep = [r for k, r in enumerate(rows) if k % 8 < 3]
    A = ([chrom[r] for r in keep], s[keep], e[keep], [name[r] for r in keep])
    gn, gl = read_genome_py(os.path.join(GOLDEN, "genome.txt"))
    auto_g = [(n, l) for n, l in zip(gn, gl) if n in auto]
    names = [n for n, _ in auto_g]
    bc, bs, be = synth.uniform([l for _, l in auto_g], 10_000, 1, 200, 2000)
    B = ([names[i] for i in bc], bs, be, [f"b{i}" for i in range(len(bs))])
    paths = []
    for tag, X in (("a", A), ("b", B)):
        p = tmp_path / f"c1_{tag}.bed"
        with open(p, "w") as f:
            for c, a, b, nm in zip(*X):
                f.write(f"{c}\t{a}\t{b}\t{nm}\n")
        paths.append(str(p))
    return A, B, paths, (gn, gl)


def ranks(*name_lists):
    from tests.util import ranked
    r = ranked(sum((list(x) for x in name_lists), []))
    return r, {v: k for k, v in r.items()}


def run_cli(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return [l.split("\t") for l in r.stdout.strip().split("\n") if l]


def test_c1_cli_against_oracle(tmp_path):
    A, B, (pa, pb), (gn, gl) = c1_inputs(tmp_path)
    assert 9000 < len(A[1]) < 11000 and len(B[1]) == 10000
    rk, inv = ranks(A[0], B[0], gn)
    ia = (np.array([rk[c] for c in A[0]], np.int32), A[1], A[2])
    ib = (np.array([rk[c] for c in B[0]], np.int32), B[1], B[2])
    # intersect (cli/Intersection.scala:41-54): every qualifying pair
    exp = oracle.intersect(ia, ib)
    want = sorted((inv[int(c)], int(s), int(e), A[3][a], B[3][b]) for c, s, e, a, b in
                  zip(exp["contig"], exp["start"], exp["end"], exp["a_row"], exp["b_row"]))
    got = sorted((c, int(s), int(e), na, nb) for c, s, e, na, nb in run_cli("intersect", pa, pb))
    assert len(want) > 20 and got == want  # ~72 expected: 1e4 x 1e4 x ~2.1 kb / 2.9 Gb
    # merge (cli/Merge.scala:36-44) and subtract (DistributedSubtract)
    m = oracle.merge(ia)
    got = [(c, int(s), int(e)) for c, s, e, _ in run_cli("merge", pa)]
    assert got == [(inv[int(c)], int(s), int(e)) for c, s, e in
                   zip(m["contig"], m["start"], m["end"])]
    sub = oracle.subtract(ia, ib)
    want = sorted((inv[int(c)], int(s), int(e), A[3][a], B[3][b] if b >= 0 else ".")
                  for c, s, e, a, b in zip(sub["contig"], sub["start"], sub["end"],
                                           sub["a_row"], sub["b_row"]))
    got = sorted((c, int(s), int(e), na, nb) for c, s, e, na, nb in run_cli("subtract", pa, pb))
    assert got == want
    # complement against the hg19 genome file (cli/Complement.scala:41-53)
    gfile = tmp_path / "genome.txt"
    gfile.write_text("".join(f"{n}\t{l}\n" for n, l in zip(gn, gl)))
    order = sorted(range(len(gn)), key=lambda i: rk[gn[i]])
    glens = [gl[i] for i in order]  # genome lengths by contig rank
    assert [rk[gn[i]] for i in order] == list(range(len(gn)))
    comp = oracle.complement(ia, glens)
    got = [(c, int(s), int(e)) for c, s, e in run_cli("complement", pa, str(gfile))]
    assert got == [(inv[int(c)], int(s), int(e)) for c, s, e in
                   zip(comp["contig"], comp["start"], comp["end"])]


# ------------------------------------------------------------------ C2
@pytest.mark.timeout(900)
def test_c2_full_size_checksum(ctx):
    sp = hg38()
    n = 100_000_000
    da, A = device_rows(ctx, sp, n, 0xA, 50, 5000)
    db, B = device_rows(ctx, sp, n, 0xB, 50, 5000)
    a, b = dset(ctx, sp, da), dset(ctx, sp, db)
    del da, db
    plan = ctx.intersect(a, b)
    got = plan.checksum()
    exp = oracle.intersect_mt(len(sp.names), A, B)
    assert plan.n == exp["n"]
    assert 1.5e10 < plan.n < 1.75e10  # E[pairs] ~ 1.63e10
    assert got == (exp["sum"], exp["xor"])
    # the bytes the benchmarked fill STORES (k_fill<false, false>, 2^31-record
    # chunks through one reusable 34 GB buffer, as bench.py), hashed from HBM
    # by a separate kernel: every stored record, not only the fill's
    # register-side checksum instantiation
    import torch
    chunk = 1 << 31
    buf = torch.empty((chunk, 4), dtype=torch.int32, device="cuda")
    hs, hx, f = 0, 0, 0
    while f < plan.n:
        k = min(chunk, plan.n - f)
        plan.fill_device(f, k, buf.data_ptr())
        s, x = ctx.pairs_checksum_device(buf.data_ptr(), k)
        hs, hx, f = (hs + s) & 0xFFFFFFFFFFFFFFFF, hx ^ x, f + k
    del buf
    assert (hs, hx) == (exp["sum"], exp["xor"])
    plan.close()
    # merge(A), merge(B): runs exact, grouping checksum of every row
    for S, X in ((a, A), (b, B)):
        res = ctx.merge(S)
        h = res.to_host()
        m = oracle.merge_mt(len(sp.names), X)
        assert_runs_equal((h["contig"], h["start"], h["end"]), (m["contig"], m["start"], m["end"]))
        ck = res.checksum()
        assert ck[2:] == (m["grp_sum"], m["grp_xor"])
        assert ck[:2] == region_checksum(m["contig"], m["start"], m["end"])


# ------------------------------------------------------------------ C3
def test_c3_pileup_merge_scaled_exact(ctx):
    # 1/50 of C3 (1e7 rows, 4e4 centres: the same rows per centre)
    sp = hg38()
    n = 10_000_000
    dev, X = device_rows(ctx, sp, n, 0xC, 150, 600, pile=(40_000, 150))
    S = dset(ctx, sp, dev)
    res = ctx.merge(S)
    h = res.to_host()
    m = oracle.merge_mt(len(sp.names), X, run_of_row=True)
    assert_runs_equal((h["contig"], h["start"], h["end"]), (m["contig"], m["start"], m["end"]))
    assert (res.run_of_row(n) == m["run_of_row"]).all()
    assert res.checksum()[2:] == (m["grp_sum"], m["grp_xor"])


@pytest.mark.timeout(900)
def test_c3_full_size(ctx):
    # BASELINE C3: 5e8 piled-up rows (2e6 centres, N(0,150) offsets, len
    # U[150,600]): exact runs, and every row's run by checksum
    sp = hg38()
    n = 500_000_000
    dev, X = device_rows(ctx, sp, n, 0xC, 150, 600, pile=(2_000_000, 150))
    S = dset(ctx, sp, dev)
    del dev
    res = ctx.merge(S)
    h = res.to_host()
    ck = res.checksum()
    m = oracle.merge_mt(len(sp.names), X)
    assert len(h["start"]) == len(m["start"]) > 100_000
    assert_runs_equal((h["contig"], h["start"], h["end"]), (m["contig"], m["start"], m["end"]))
    assert ck[2:] == (m["grp_sum"], m["grp_xor"])


# ------------------------------------------------------------------ C4
@pytest.mark.timeout(600)
def test_c4_bitset_hg38(ctx):
    sp = hg38()
    n = 10_000_000
    da, A = device_rows(ctx, sp, n, 0xD, 50, 500)
    db, B = device_rows(ctx, sp, n, 0xE, 50, 500)
    ba, bb = dbits(ctx, sp, da), dbits(ctx, sp, db)  # the C4 path: binned paint
    # complement(merge(A)) vs hg38 == bitset NOT (coalesced: A.4)
    lens = sp.lengths.tolist()
    comp = ctx.bitset_runs(1, ba).to_host()
    Ai = (A[0], A[1].astype(np.int64), A[2].astype(np.int64))
    exp = oracle.complement(Ai, lens)
    assert_runs_equal(coalesce(comp["contig"], comp["start"], comp["end"]),
                      coalesce(exp["contig"], exp["start"], exp["end"]))
    # merge(A) \ merge(B) per base == set-mode subtract of the merged runs
    ma = oracle.merge_mt(len(lens), A)
    mb = oracle.merge_mt(len(lens), B)
    assert ba.popcount() == int((ma["end"] - ma["start"]).sum())
    diff = ctx.bitset_runs(3, ba, bb).to_host()
    exp = oracle.subtract((ma["contig"], ma["start"], ma["end"]),
                          (mb["contig"], mb["start"], mb["end"]), 0, oracle.SUB_SET)
    assert_runs_equal(coalesce(diff["contig"], diff["start"], diff["end"]),
                      coalesce(exp["contig"], exp["start"], exp["end"]))


# ------------------------------------------------------------------ C5
def fold_and(n_contigs, merged):
    """A.4: the fold of intersect over merged operands (disjoint sorted runs)"""
    cur = merged[0]
    for m in merged[1:]:
        ix = oracle.intersect_mt(n_contigs, (cur["contig"], cur["start"], cur["end"]),
                                 (m["contig"], m["start"], m["end"]), records=True)
        cur = {k: ix[k] for k in ("contig", "start", "end")}
    return cur


@pytest.mark.timeout(600)
def test_c5_eight_way_and_density(ctx):
    sp = hg38(8)
    per = 125_000_000 // 8
    merged, bits, devs = [], [], []
    for i in range(8):
        dev, X = device_rows(ctx, sp, per, 0x50 + i, 10, 40)
        bits.append(dbits(ctx, sp, dev))  # unsorted rows -> binned paint, per set
        merged.append(oracle.merge_mt(len(sp.names), X))
        devs.append(dev)
    got = ctx.bitset_and(bits).to_host()
    exp = fold_and(len(sp.names), merged)
    g = coalesce(got["contig"], got["start"], got["end"])
    assert_runs_equal(g, coalesce(exp["contig"], exp["start"], exp["end"]))
    # the bench's path: the 8 sets binned and painted-and-ANDed in one kernel
    fused = ctx.bitset_and_from_device(
        sp, [(d[0].numel(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()) for d in devs])
    f = ctx.bitset_runs(0, fused).to_host()
    assert_runs_equal((f["contig"], f["start"], f["end"]), (got["contig"], got["start"], got["end"]))
    cov = int((g[2] - g[1]).sum())
    assert 0.01 < cov / sum(sp.lengths) < 0.05  # 8-way ~2.7% of the genome


@pytest.mark.timeout(600)
def test_c5_optimistic_binning_and_sorted_fallback(monkeypatch, capfd):
    # With LIME_BIN_OPTIMISTIC=1 bit-per-base builds bin rows without a count
    # pass when the window's uniform density fills each (bin, chunk) region
    # (mean + 6 sigma slots): C5's shape, here on hg38/8 with 3 x 1.5625e7
    # rows.  (Opt-in: on C5 it measured no faster than the counted path.)  The same rows in
    # SORTED order (a sorted BED file) put each chunk's rows in one or two
    # bins: the regions overflow, the set is binned again through the counted
    # path, and the results are unchanged -- through the k-way AND (pipelined
    # sets) and the one-set build, against the oracle fold (A.4).  A fresh
    # context: after an overflow the context prefers the counted path for its
    # next builds (lime_ctx.bin_pessimism), which must not leak into other tests
    import torch

    import lime_amd
    monkeypatch.setenv("LIME_TRACE_BINNING", "1")
    monkeypatch.setenv("LIME_BIN_OPTIMISTIC", "1")
    c = lime_amd.Context(0)
    try:
        sp = hg38(8)
        per = 125_000_000 // 8
        devs, merged = [], []
        for i in range(3):
            dev, X = device_rows(c, sp, per, 0x70 + i, 10, 40)
            devs.append(dev)
            merged.append(oracle.merge_mt(len(sp.names), X))
        exp = fold_and(len(sp.names), merged)
        want = coalesce(exp["contig"], exp["start"], exp["end"])

        def and_runs(ds):
            b = c.bitset_and_from_device(
                sp, [(d[0].numel(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()) for d in ds])
            r = c.bitset_runs(0, b).to_host()
            b.close()
            return coalesce(r["contig"], r["start"], r["end"])
        capfd.readouterr()
        assert_runs_equal(and_runs(devs), want)
        log = capfd.readouterr().err
        assert log.count("optimistic") == 3 and "overflow" not in log, log
        # the same rows sorted by (contig, start)
        sdevs = []
        for d in devs:
            key = d[0].to(torch.int64) * (1 << 32) + d[1].to(torch.int64)
            o = torch.argsort(key)
            sdevs.append(tuple(x[o].contiguous() for x in d))
        torch.cuda.synchronize()
        assert_runs_equal(and_runs(sdevs), want)
        log = capfd.readouterr().err
        assert "overflow" in log and "counted" in log, log
        # one set through the single-set build (bin_set), sorted: counted first
        # now, then (pessimism spent) optimistic again, overflowing again
        one = merged[0]
        w1 = coalesce(one["contig"], one["start"], one["end"])
        for _ in range(2):
            b = dbits(c, sp, sdevs[0])
            r = c.bitset_runs(0, b).to_host()
            b.close()
            assert_runs_equal(coalesce(r["contig"], r["start"], r["end"]), w1)
    finally:
        c.close()


@pytest.mark.timeout(900)
def test_c2_subtract_full_size(ctx):
    # DistributedSubtract (Subtract.scala:91-116) on C2's inputs at full size,
    # both modes: region count + region checksum == the contig-sharded oracle
    # (lo_subtract_mt).  At C2's depth (~160x coverage by B) only a handful
    # of A's bases escape B: 16 remnants per mode on the GPU box
    sp = hg38()
    n = 100_000_000
    da, A = device_rows(ctx, sp, n, 0xA, 50, 5000)
    db, B = device_rows(ctx, sp, n, 0xB, 50, 5000)
    a, b = dset(ctx, sp, da), dset(ctx, sp, db)
    del da, db
    for mode in (oracle.SUB_LIME, oracle.SUB_SET):
        res = ctx.subtract(a, b, 0, mode)
        ck = res.checksum()
        exp = oracle.subtract_mt(len(sp.names), A, B, 0, mode)
        assert res.n == exp["n"] > 0
        assert ck[:2] == (exp["sum"], exp["xor"])
        res.close()
