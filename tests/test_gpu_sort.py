"""The partition-and-sort stage (ADAM
repartitionAndSort, cli/Intersection.scala:42-43) against a numpy stable
sort, on inputs that take every path of lime_amd/csrc/sort.hip:

  - the bucketed sort (two digit passes of 8 + 8, 9 + 8 or 9 + 9 bits on
    bits [L, 32) of the global start, then every 2^L-base bucket sorted in
    LDS): buckets of a few rows, of ~2k rows (k_local_small), ~2.7k
    (k_local_keys mid), ~6-11k (k_local_keys wide), with sub-bins past SMAX
    and buckets past 16k rows (k_local_big: ranked passes, the workgroup-wide
    radix over global memory);
  - the digit passes (spans within 16 bits, sets of few rows per bucket,
    sets past LAVG rows per bucket: both sides of that switch at full size
    over hg38, C3-shaped pile-ups, giant piles, global rows);
  - the packed second bucket pass (one word per row, gs mod 2^L and the
    width) with the bucket starts from its histogram's partial counts,
    first-digit regions crowded into a few tiles, widths at the u16 limit;
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


@pytest.mark.parametrize("wmax", [65_535, 65_536])
def test_digit_pass_u16_widths(ctx, wmax):
    # digit-pass sets without zero-width rows carry u16 widths between the
    # first and the last pass when every width is < 2^16: widths up to the
    # limit (65,535 present) and one row past it (the u32 passes), host rows
    # and global rows with caller row ids
    import torch
    rng = np.random.default_rng(wmax)
    L = 40_000_000
    sp = _space([L, 5_000_000])
    n = 400_000
    c = (rng.random(n) < 0.2).astype(np.int32)
    s = (rng.random(n) * (np.array([L, 5_000_000])[c] - 70_000)).astype(np.int64)
    w = rng.integers(1, 65_536, n)
    w[rng.integers(0, n, 50)] = 65_535
    w[rng.integers(0, n, 50)] = 1
    w[7] = wmax
    e = s + w
    d = rng.integers(0, n, 2000)
    s[d[:1000]], e[d[:1000]], c[d[:1000]] = s[d[1000:]], e[d[1000:]], c[d[1000:]]
    _check_host_set(ctx, sp, c, s, e)
    off = sp.offsets[:-1]
    gs, ge = (off[c] + s).astype(np.uint32), (off[c] + e).astype(np.uint32)
    rows = rng.permutation(3 * n)[:n].astype(np.uint32)
    tg = [torch.tensor(x.view(np.int32), device="cuda") for x in (gs, ge, rows)]
    got = ctx.set_from_global(sp, n, *(t.data_ptr() for t in tg)).to_host()
    order = _expected(gs.astype(np.int64), ge.astype(np.int64))
    assert (got["row"] == rows[order]).all()
    assert (got["start"] == s[order]).all() and (got["end"] == e[order]).all()


def _check_device_order(ctx, sp, n, c, s, e):
    """the set built from device rows (c, s, e) is in canonical order (gs,
    zero-width first, input row), its row ids a permutation and every row's
    coordinates those of its input row -- checked on the device at full size"""
    import torch
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


def _hg38():
    from lime_amd import synth
    return Space(list(synth.HG38.keys()), list(synth.HG38.values()))


def _synth(ctx, sp, n, seed, lo, hi, pile=None):
    import torch
    c, s, e = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    if pile:
        ctx.synth_pileup(sp, n, seed, pile[0], pile[1], lo, hi, c.data_ptr(), s.data_ptr(),
                         e.data_ptr())
    else:
        ctx.synth_uniform(sp, n, seed, lo, hi, c.data_ptr(), s.data_ptr(), e.data_ptr())
    torch.cuda.synchronize()
    return c, s, e


# hg38: sbits 32, 47,125 buckets of 65,536 bases.  LAVG (2304) rows per
# bucket switch a set from k_local_small to the keys kernels (sort.hip); both
# sides of the switch are exercised at full size.
_BUCKETS_HG38 = 47_125


@pytest.mark.parametrize("n", [2304 * _BUCKETS_HG38 - 1_000_000, 2304 * _BUCKETS_HG38 + 1_000_000])
def test_bucketed_sort_switch_point(ctx, n):
    # uniform rows over hg38, len U[0, 60] (zero-width rows included): below
    # the switch two 8-bit passes and k_local_small, above it k_local_keys
    sp = _hg38()
    c, s, e = _synth(ctx, sp, n, 0x5A, 0, 60)
    _check_device_order(ctx, sp, n, c, s, e)


def test_bucketed_sort_packed_partials(ctx):
    # the packed second pass places every bucket from k_hist_part's partial
    # counts.  Here 2.05e6 rows over hg38: 2e6 of them in one pile at one
    # start (one first digit, one bucket through k_local_big's workgroup
    # radix), the rest spread thin, so the first-digit regions of those few
    # rows crowd into a handful of pass-1 tiles: a tile sees many regions
    # start (the partial rounds of 16 first digits each), and most (d2, D)
    # buckets are empty (their starts from the scanned counts alone).
    # Widths up to 65,535 (the packed word's limit) and zero-width rows.
    rng = np.random.default_rng(61)
    sp = _hg38()
    lens = np.array(sp.lengths)
    n_pile, n_thin = 2_000_000, 50_000
    big = np.flatnonzero(lens > 1_000_000)  # (not chrM: room for 65,535-base rows)
    c = np.concatenate([np.full(n_pile, 2, np.int32),
                        big[rng.integers(0, len(big), n_thin)].astype(np.int32)])
    s = np.concatenate([np.full(n_pile, 1_234_567, np.int64),
                        (rng.random(n_thin) * (lens[c[n_pile:]] - 70_000)).astype(np.int64)])
    w = rng.integers(0, 600, len(c))
    w[rng.integers(0, len(c), 500)] = 65_535
    w[rng.integers(0, len(c), 20_000)] = 0
    e = s + w
    perm = rng.permutation(len(c))
    _check_host_set(ctx, sp, c[perm], s[perm], e[perm])


def test_bucketed_sort_dense_buckets(ctx):
    # C3's shape at 2e8 rows: pile-ups (8e5 centres over hg38, N(0,150), len
    # U[150,600]) averaging ~4.2k rows per 65536-base bucket: the wide keys
    # kernel (C3 itself: ~10.6k)
    sp = _hg38()
    n = 200_000_000
    c, s, e = _synth(ctx, sp, n, 0x3C, 150, 600, pile=(800_000, 150))
    _check_device_order(ctx, sp, n, c, s, e)


def test_digit_pass_sort_giant_piles(ctx):
    # 1.2e8 rows over hg38 (~2.5k per 2^16-base bucket: the mid keys kernel)
    # with piles of 2.5k, 9k, 40k and 150k rows at single positions,
    # zero-width rows and duplicates among them: sub-bins past SMAX and
    # buckets past the caps (k_local_big's ranked passes and its radix over
    # global memory), stable at every pile
    import torch
    sp = _hg38()
    n = 120_000_000
    c, s, e = _synth(ctx, sp, n, 0x61, 50, 500)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    for k, (size, pos) in enumerate([(2_500, 1_000_000), (9_000, 5_000_000),
                                     (40_000, 9_000_100), (150_000, 70_000_000)]):
        idx = torch.randperm(n, device="cuda", generator=g)[:size]
        c[idx] = 1 + k
        s[idx] = pos + torch.randint(0, 3000, (size,), device="cuda", generator=g,
                                     dtype=torch.int32)
        w = torch.randint(0, 400, (size,), device="cuda", generator=g, dtype=torch.int32)
        w[torch.rand(size, device="cuda", generator=g) < 0.1] = 0
        e[idx] = s[idx] + w
    torch.cuda.synchronize()
    _check_device_order(ctx, sp, n, c, s, e)


def test_digit_pass_sort_global(ctx):
    # global-coordinate rows with the caller's row ids (1.15e8 rows over hg38:
    # the bucketed passes from the caller's (gs, ge, row), ROWS_LOAD): ties
    # keep INPUT order, rows carried through
    import torch
    sp = _hg38()
    n = 115_000_000
    c, s, e = _synth(ctx, sp, n, 0x62, 0, 40)
    off = torch.tensor(sp.offsets[:-1].astype(np.int64), device="cuda")
    gs = (off[c.to(torch.int64)] + s.to(torch.int64)).to(torch.int64)
    ge = (off[c.to(torch.int64)] + e.to(torch.int64)).to(torch.int64)
    rows = torch.arange(n, device="cuda", dtype=torch.int64) * 3 + 7
    t32 = [torch.where(x >= 2**31, x - 2**32, x).to(torch.int32) for x in (gs, ge, rows)]
    torch.cuda.synchronize()  # (torch's stream is not the engine's)
    S = ctx.set_from_global(sp, n, *(t.data_ptr() for t in t32))
    og, oe, orow = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    S.copy_rows_device(0, n, og.data_ptr(), oe.data_ptr(), orow.data_ptr())
    torch.cuda.synchronize()
    S.close()
    g64, e64, r64 = (x.to(torch.int64) & 0xFFFFFFFF for x in (og, oe, orow))
    key = g64 * 2 + (e64 > g64).to(torch.int64)
    assert bool((key[1:] >= key[:-1]).all())
    tie = key[1:] == key[:-1]
    assert bool((r64[1:][tie] > r64[:-1][tie]).all())
    i = (r64 - 7) // 3
    assert bool(((r64 - 7) % 3 == 0).all())
    assert bool((torch.sort(i).values == torch.arange(n, device="cuda")).all())
    assert bool((g64 == gs[i]).all()) and bool((e64 == ge[i]).all())


# The bucketed sort's local kernels and wider digit passes over a span of
# 2^27 + 1 (sbits 28):
#   mid:   9e7 rows, ~2.7k per 2^12-base bucket under two 8-bit passes
#          (k_local_keys 512 x 12);
#   wide:  2.2e8 rows, ~6.7k per bucket (k_local_keys 1024 x 16);
#   nine:  4e8 rows average past LAVG_W per 2^12-base bucket, so the passes
#          take 17 bits (9 + 8) and the buckets are 2^11 bases (~6.1k rows),
#          with widths past 2^16 (u32 ends through the 9-bit pass) as global
#          rows with the caller's row ids;
#   piles: the wide shape with piles that overflow it (a position holding 60
#          rows: a sub-bin past SMAX; 40,000 rows in one bucket: past its
#          16,384-row cap, the workgroup radix over global memory) and 8,000
#          rows in one bucket.
_W18 = 1 << 27


@pytest.mark.parametrize("case", ["mid", "wide", "nine_global", "piles"])
def test_bucketed_sort_local_shapes(ctx, case):
    import torch
    sp = _space([_W18])
    n = {"mid": 90_000_000, "wide": 220_000_000, "nine_global": 400_000_000,
         "piles": 220_000_000}[case]
    hi = 70_000 if case == "nine_global" else 60
    c, s, e = _synth(ctx, sp, n, 0x918, 0, hi)
    if case == "piles":
        g = torch.Generator(device="cuda")
        g.manual_seed(18)
        for size, pos, spread in [(60, 5_000_000, 1), (8_000, 9_000_000, 1000),
                                  (40_000, 70_000_000, 1000)]:
            idx = torch.randperm(n, device="cuda", generator=g)[:size]
            s[idx] = pos + torch.randint(0, spread, (size,), device="cuda", generator=g,
                                         dtype=torch.int32)
            w = torch.randint(0, 300, (size,), device="cuda", generator=g, dtype=torch.int32)
            w[torch.rand(size, device="cuda", generator=g) < 0.1] = 0
            e[idx] = s[idx] + w
        torch.cuda.synchronize()
    if case != "nine_global":
        _check_device_order(ctx, sp, n, c, s, e)
        return
    # global rows with caller row ids: ties keep INPUT order
    rows = torch.arange(n, device="cuda", dtype=torch.int64) * 5 + 3
    r32 = torch.where(rows >= 2**31, rows - 2**32, rows).to(torch.int32)
    del rows
    torch.cuda.synchronize()
    S = ctx.set_from_global(sp, n, s.data_ptr(), e.data_ptr(), r32.data_ptr())
    del r32
    og, oe, orow = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    S.copy_rows_device(0, n, og.data_ptr(), oe.data_ptr(), orow.data_ptr())
    torch.cuda.synchronize()
    S.close()
    g64, e64, r64 = (x.to(torch.int64) & 0xFFFFFFFF for x in (og, oe, orow))
    del og, oe, orow
    key = g64 * 2 + (e64 > g64).to(torch.int64)
    assert bool((key[1:] >= key[:-1]).all())
    tie = key[1:] == key[:-1]
    assert bool((r64[1:][tie] > r64[:-1][tie]).all())
    del key, tie
    i = (r64 - 3) // 5
    assert bool(((r64 - 3) % 5 == 0).all())
    assert bool((torch.sort(i).values == torch.arange(n, device="cuda")).all())
    assert bool((g64 == s.to(torch.int64)[i]).all()) and bool((e64 == e.to(torch.int64)[i]).all())
    assert int((e64 - g64).max()) >= 65_536


def test_digit_pass_pileups_ident_to16(ctx):
    # pile-up keys through the digit passes' first pass exactly as round 4's
    # unrecorded fault had them: caller rows (ROWS_IDENT: row = position)
    # turned into u16 widths (EW_TO16), then EW_16 / EW_FROM16.  1.2e6 rows
    # in 5,000 centres over hg38 average ~25 rows per 2^16-base bucket, below
    # the bucketed sort's LMIN (32), so the four digit passes run; piles of
    # ~240 rows per centre, zero-width rows among them
    import torch
    sp = _hg38()
    n = 1_200_000
    c, s, e = _synth(ctx, sp, n, 0x7E, 150, 600, pile=(5_000, 150))
    z = torch.rand(n, device="cuda") < 0.02
    e[z] = s[z]
    torch.cuda.synchronize()
    _check_device_order(ctx, sp, n, c, s, e)
