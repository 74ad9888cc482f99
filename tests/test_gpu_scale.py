"""north_star's 1B-interval target and full-size C5 (SURVEY.md 8(d)
"Verification at scale"): the HIP engine through the C-ABI against the
contig-sharded oracle drivers, by count plus order-independent checksum
(the outputs are too large to compare record by record).

  1e9-row merge / complement   1e9 ChIP-seq-like pile-up rows (4e6 centres,
      N(0,150) offsets, len U[150,600]): merge runs exact and the checksum of
      every row's run (SetTheory.scala:208-225); complement gaps by count and
      region checksum (Complement.scala:59-128)
  2 x 5e8 intersect / subtract  uniform over hg38, len U[10,40] (~4e9 pairs):
      pair count + pair checksum, of the fill's register side and of every
      record it stores (Intersection.scala:58-69); subtract in both modes by
      count + region checksum (Subtract.scala:91-116)
  sparse-B subtract  1e7 long left rows (len U[1000,10000]) minus 3e7 short
      right rows (len U[10,40]): ~50 blocks per left row, ~5e8 remnants in
      lime mode (Subtract.scala:103-114's per-block emission at volume)
  C5 at full size  8 x 1.25e8 rows over hg38, len U[10,40]: the fused k-way
      paint-AND (the bench's path) == the oracle fold of intersect over the
      merged operands (Appendix A.4), runs exact

Inputs come from the device generator, anchored to the numpy restatement;
the oracle reads host copies.  Progress lines are printed (run with -s) so a
long oracle call is not mistaken for a hang."""
import time

import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_configs import assert_runs_equal, coalesce, device_rows, dset, hg38

pytestmark = pytest.mark.gpu

T0 = time.time()


def say(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", flush=True)


# --------------------------------------------------------- 1e9 pile-up rows
@pytest.fixture(scope="module")
def pile_1b(ctx):
    sp = hg38()
    n = 1_000_000_000
    say("1e9 pile-up rows: generating")
    dev, host = device_rows(ctx, sp, n, 0x1B, 150, 600, pile=(4_000_000, 150))
    S = dset(ctx, sp, dev)
    del dev
    say("1e9 pile-up rows: sorted set built")
    yield sp, S, host
    S.close()


@pytest.mark.timeout(600)
def test_1b_merge(ctx, pile_1b):
    sp, S, X = pile_1b
    res = ctx.merge(S)
    h = res.to_host()
    ck = res.checksum()
    say(f"merge: {res.n} runs on the device; oracle")
    m = oracle.merge_mt(len(sp.names), X)
    say("merge: oracle done")
    assert len(h["start"]) == len(m["start"]) > 500_000  # ~7.3e5 pile-up clusters
    assert_runs_equal((h["contig"], h["start"], h["end"]), (m["contig"], m["start"], m["end"]))
    assert ck[2:] == (m["grp_sum"], m["grp_xor"])  # every row's run
    res.close()


@pytest.mark.timeout(600)
def test_1b_complement(ctx, pile_1b):
    sp, S, X = pile_1b
    res = ctx.complement(sp, S)
    ck = res.checksum()
    say(f"complement: {res.n} gaps on the device; oracle")
    e = oracle.complement_mt(sp.lengths, X)
    say("complement: oracle done")
    assert res.n == e["n"] > 500_000  # ~7.3e5 gaps between the pile-up clusters
    assert ck[:2] == (e["sum"], e["xor"])
    res.close()


# ------------------------------------------------- 2 x 5e8 uniform rows
@pytest.fixture(scope="module")
def pair_1b(ctx):
    sp = hg38()
    n = 500_000_000
    say("2 x 5e8 uniform rows: generating")
    da, A = device_rows(ctx, sp, n, 0x1A, 10, 40)
    db, B = device_rows(ctx, sp, n, 0x1C, 10, 40)
    a, b = dset(ctx, sp, da), dset(ctx, sp, db)
    del da, db
    say("2 x 5e8 uniform rows: sorted sets built")
    yield sp, a, b, A, B
    a.close()
    b.close()


@pytest.mark.timeout(600)
def test_1b_intersect(ctx, pair_1b):
    sp, a, b, A, B = pair_1b
    plan = ctx.intersect(a, b)
    got = plan.checksum()
    say(f"intersect: {plan.n} pairs on the device; oracle")
    exp = oracle.intersect_mt(len(sp.names), A, B)
    say("intersect: oracle done")
    assert plan.n == exp["n"]
    assert 3.5e9 < plan.n < 4.5e9  # E = n^2 (25 + 25) / G ~ 4.0e9
    assert got == (exp["sum"], exp["xor"])
    # the bytes the fill STORES on this sparse plan (~4 pairs per owner, the
    # tile-commit-bound shape), 2^31-record chunks through one reusable
    # buffer as bench_extra's b1_pair line, hashed from HBM by a separate
    # kernel: every stored record, not the fill's register-side checksum
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
    say("intersect: stored records hashed")
    assert (hs, hx) == (exp["sum"], exp["xor"])
    plan.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [oracle.SUB_LIME, oracle.SUB_SET])
def test_1b_subtract(ctx, pair_1b, mode):
    sp, a, b, A, B = pair_1b
    res = ctx.subtract(a, b, 0, mode)
    ck = res.checksum()
    say(f"subtract mode {mode}: {res.n} regions on the device; oracle")
    exp = oracle.subtract_mt(len(sp.names), A, B, 0, mode)
    say("subtract: oracle done")
    assert res.n == exp["n"] > 1e6  # lime mode: ~7.4e7 regions
    assert ck[:2] == (exp["sum"], exp["xor"])
    res.close()


# ------------------------------------------- sparse B from long left rows
@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [oracle.SUB_LIME, oracle.SUB_SET])
def test_sparse_b_subtract_long_rows(ctx, mode):
    # every left row is cut by ~50 separate B rows: many blocks per row and a
    # remnant per block (lime mode: Subtract.scala:103-114; set mode: the
    # pieces of a minus the union of its hits)
    sp = hg38()
    da, A = device_rows(ctx, sp, 10_000_000, 0x5A, 1000, 10000)
    db, B = device_rows(ctx, sp, 30_000_000, 0x5B, 10, 40)
    a, b = dset(ctx, sp, da), dset(ctx, sp, db)
    del da, db
    res = ctx.subtract(a, b, 0, mode)
    ck = res.checksum()
    say(f"sparse-B subtract mode {mode}: {res.n} regions on the device; oracle")
    exp = oracle.subtract_mt(len(sp.names), A, B, 0, mode)
    say("sparse-B subtract: oracle done")
    assert res.n == exp["n"] > 2e8  # ~50 pieces per left row
    assert ck[:2] == (exp["sum"], exp["xor"])
    for h in (res, a, b):
        h.close()


# ------------------------------------------------------- C5 at full size
def fold_and(n_contigs, merged):
    """A.4: the fold of intersect over merged operands (disjoint sorted runs)"""
    cur = merged[0]
    for m in merged[1:]:
        ix = oracle.intersect_mt(n_contigs, (cur["contig"], cur["start"], cur["end"]),
                                 (m["contig"], m["start"], m["end"]), records=True)
        cur = {k: ix[k] for k in ("contig", "start", "end")}
    return cur


@pytest.mark.timeout(600)
def test_c5_full_size(ctx):
    # BASELINE C5: 8 x 1.25e8 rows (len U[10,40], seeds 0x50..0x57) over the
    # whole hg38, the bench's fused paint-AND, against the oracle fold
    sp = hg38()
    per = 125_000_000
    devs, merged = [], []
    for i in range(8):
        dev, X = device_rows(ctx, sp, per, 0x50 + i, 10, 40)
        devs.append(dev)
        merged.append(oracle.merge_mt(len(sp.names), X))
        del X
        say(f"C5: set {i} generated and merged by the oracle")
    fused = ctx.bitset_and_from_device(
        sp, [(d[0].numel(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()) for d in devs])
    got = ctx.bitset_runs(0, fused).to_host()
    fused.close()
    del devs
    say(f"C5: {len(got['start'])} runs on the device; oracle fold")
    exp = fold_and(len(sp.names), merged)
    say("C5: oracle fold done")
    assert len(got["start"]) > 10_000_000  # ~1.39e7 runs at C5's density
    assert_runs_equal(coalesce(got["contig"], got["start"], got["end"]),
                      coalesce(exp["contig"], exp["start"], exp["end"]))
