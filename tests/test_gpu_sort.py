"""The partition-and-sort stage (ADAM
repartitionAndSort, cli/Intersection.scala:42-43) against a numpy stable
sort, on inputs that take every path of lime_amd/csrc/sort.hip:

  - the bucketed sort (two 8-bit digit passes on bits [L, L + 16) of the
    global start, then every 2^L-base bucket sorted in LDS): buckets of a few
    rows, buckets of ~2-4k rows (512-thread kernel), of 4k-16k rows
    (1024-thread kernel) and past 16k rows (the workgroup-wide radix over
    global memory);
  - the digit passes (spans within 16 bits, sets of few rows per bucket;
    sets averaging more than LAVG rows per bucket run through the 1e9-row
    tests of tests/test_gpu_scale.py);
  - host, device and global-coordinate inputs, zero-width rows, exact
    duplicates, rows already in order.

Canonical order: (global start, zero-width first, input order); the row id
of a host / device set is the input index."""
import numpy as np
import pytest

from lime_amd import Space

pytestmark = pytest.mark.gpu


def _expected(gs, ge):
    """stable order by (gs, zero-width first): input order breaks ties"""
    nz = (ge > gs).astype(np.int64)
    return np.lexsort((np.arange(len(gs)), nz, gs))


def _space(lengths):
    return Space([f"c{i:02d}" for i in range(len(lengths))], lengths)


def _check_host_set(ctx, sp, c, s, e):
    h = ctx.set_from_host(sp, c, s, e).to_host()
    off = sp.offsets[:-1]
    gs = off[c] + s
    ge = off[c] + e
    order = _expected(gs, ge)
    assert (h["row"] == order).all()
    assert (h["start"] == s[order]).all() and (h["end"] == e[order]).all()
    assert (h["contig"] == c[order]).all()


def _rows(rng, n, lo, hi, width_max, zero_frac=0.0, dup_frac=0.0):
    s = rng.integers(lo, hi, n)
    e = s + rng.integers(1, width_max, n)
    z = rng.random(n) < zero_frac
    e[z] = s[z]
    d = np.flatnonzero(rng.random(n) < dup_frac)
    if len(d) > 1:  # exact duplicates of other rows
        src = rng.integers(0, n, len(d))
        s[d], e[d] = s[src], e[src]
    return s, e


@pytest.mark.parametrize("seed", [1, 2])
def test_bucketed_sort_uniform(ctx, seed):
    # a 690 Mb span, ~60 rows per bucket: every bucket in the small kernel
    rng = np.random.default_rng(seed)
    lens = [248_956_422, 242_193_529, 198_295_559, 16_569]
    sp = _space(lens)
    n = 2_500_000
    c = rng.integers(0, len(lens), n).astype(np.int32)
    s = (rng.random(n) * (np.array(lens)[c] - 6000)).astype(np.int64)
    e = s + rng.integers(0, 5000, n)
    z = rng.random(n) < 0.05
    e[z] = s[z]
    _check_host_set(ctx, sp, c, s, e)


def test_bucketed_sort_every_bucket_shape(ctx):
    # 50 Mb contig: L = 10 (1024-base buckets).  Background rows keep the
    # average bucket small; three pile-ups make buckets of ~2.5k rows (small
    # kernel), ~9k rows (the 1024-thread LDS kernel) and ~40k rows (the
    # workgroup radix over global memory), with zero-width rows and duplicates
    rng = np.random.default_rng(7)
    L = 50_000_000
    sp = _space([L])
    parts = [_rows(rng, 2_500_000, 0, L - 10_000, 3000, 0.05, 0.02),
             _rows(rng, 2_500, 1_000_000, 1_000_900, 300, 0.1, 0.3),
             _rows(rng, 9_000, 2_000_000, 2_001_000, 300, 0.1, 0.3),
             _rows(rng, 40_000, 3_000_050, 3_001_000, 300, 0.1, 0.3)]
    s = np.concatenate([p[0] for p in parts])
    e = np.concatenate([p[1] for p in parts])
    perm = rng.permutation(len(s))
    s, e = s[perm], e[perm]
    c = np.zeros(len(s), np.int32)
    _check_host_set(ctx, sp, c, s, e)


def test_bucketed_sort_device_and_global(ctx):
    import torch
    rng = np.random.default_rng(11)
    L = 200_000_000
    sp = _space([L, 1000])
    n = 2_000_000
    s, e = _rows(rng, n, 0, L - 5000, 5000, 0.05, 0.05)
    c = np.zeros(n, np.int32)
    dc = torch.tensor(c, device="cuda")
    ds = torch.tensor(s.astype(np.int32), device="cuda")
    de = torch.tensor(e.astype(np.int32), device="cuda")
    h = ctx.set_from_device(sp, n, dc.data_ptr(), ds.data_ptr(), de.data_ptr()).to_host()
    order = _expected(s, e)
    assert (h["row"] == order).all() and (h["start"] == s[order]).all()
    # global coordinates with caller row ids: ties keep INPUT order
    rows = rng.permutation(10 * n)[:n].astype(np.uint32)
    gs, ge = s.astype(np.uint32), e.astype(np.uint32)
    tg = [torch.tensor(x.view(np.int32), device="cuda") for x in (gs, ge, rows)]
    S = ctx.set_from_global(sp, n, *(t.data_ptr() for t in tg))
    got = S.to_host()
    assert (got["row"] == rows[order]).all()
    assert (got["start"] == s[order]).all() and (got["end"] == e[order]).all()


def test_sorted_input_and_digit_pass_sets(ctx):
    rng = np.random.default_rng(3)
    # already in canonical order: no passes, rows = positions
    L = 30_000_000
    sp = _space([L])
    s, e = _rows(rng, 2_000_000, 0, L - 2000, 2000, 0.1, 0.0)
    o = _expected(s, e)
    _check_host_set(ctx, sp, np.zeros(len(s), np.int32), s[o], e[o])
    # too few rows per bucket: the digit passes
    s, e = _rows(rng, 300_000, 0, L - 2000, 2000, 0.1, 0.1)
    _check_host_set(ctx, sp, np.zeros(len(s), np.int32), s, e)
    # a span within 16 bits: the digit passes
    sp2 = _space([60_000])
    s, e = _rows(rng, 300_000, 0, 60_000 - 100, 100, 0.1, 0.1)
    _check_host_set(ctx, sp2, np.zeros(len(s), np.int32), s, e)


def test_bucketed_sort_dense_buckets(ctx):
    # C3's shape at 2e8 rows: pile-ups (8e5 centres over hg38, N(0,150), len
    # U[150,600]) averaging ~4.2k rows per 65536-base bucket: denser than the
    # bucketed sort takes, so the four digit passes.  Checked on the device at
    # full size: canonical order (gs, zero-width first, input row), the row
    # ids a permutation, every row's coordinates those of its input row.
    import torch

    from lime_amd import synth
    sp = Space(list(synth.HG38.keys()), list(synth.HG38.values()))
    n = 200_000_000
    c = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    e = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.synth_pileup(sp, n, 0x3C, 800_000, 150, 150, 600, c.data_ptr(), s.data_ptr(), e.data_ptr())
    torch.cuda.synchronize()
    S = ctx.set_from_device(sp, n, c.data_ptr(), s.data_ptr(), e.data_ptr())
    gs, ge, row = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    S.copy_rows_device(0, n, gs.data_ptr(), ge.data_ptr(), row.data_ptr())
    torch.cuda.synchronize()
    S.close()
    off = torch.tensor(sp.offsets[:-1].astype(np.int64), device="cuda")
    g64 = gs.to(torch.int64) & 0xFFFFFFFF
    e64 = ge.to(torch.int64) & 0xFFFFFFFF
    key = g64 * 2 + (e64 > g64).to(torch.int64)
    assert bool((key[1:] >= key[:-1]).all())
    tie = key[1:] == key[:-1]
    r64 = row.to(torch.int64) & 0xFFFFFFFF
    assert bool((r64[1:][tie] > r64[:-1][tie]).all())
    assert bool((torch.sort(r64).values == torch.arange(n, device="cuda")).all())
    cin = c.to(torch.int64)[r64]
    assert bool((g64 == off[cin] + s.to(torch.int64)[r64]).all())
    assert bool((e64 == off[cin] + e.to(torch.int64)[r64]).all())
