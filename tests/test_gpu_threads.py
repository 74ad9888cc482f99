"""Reentrancy of the C-ABI (SURVEY.md 8(b) "Threading"): Spark runs the
per-partition body on N executor threads, each with its own deserialized
operator and mutable cache (SetTheory.scala:83).  Here N host threads each
own a lime_ctx and run intersect, merge and subtract concurrently (ctypes
drops the GIL around every engine call); every result must equal the oracle.
Sets are bound to their context: an operator called with another context's
set is rejected (LIME_ERR_ARG) instead of reading or caching state across
contexts."""
import threading

import numpy as np
import pytest

from lime_amd import Context, LimeError, SUBTRACT_LIME, SUBTRACT_SET, Space
from oracle import oracle
from tests.util import as_sorted_tuples, random_sets

pytestmark = pytest.mark.gpu

NAMES = ["t0", "t1", "t2"]


def _job(k, out):
    try:
        rng = np.random.default_rng(900 + k)
        A, B = random_sets(rng, 6000, 5000, n_contigs=3, contig_len=50000, max_len=600,
                           zero_frac=0.05, dup_frac=0.05, book_frac=0.1)
        ctx = Context(0)
        sp = Space(NAMES, [50000] * 3)
        res = {}
        for rep in range(3):  # repeated calls reuse each context's pool
            a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
            plan = ctx.intersect(a, b)
            p = plan.fill_host()
            res["pairs"] = as_sorted_tuples({"contig": A[0][p["a_row"]], "start": p["start"],
                                             "end": p["end"], "a_row": p["a_row"],
                                             "b_row": p["b_row"]})
            m = ctx.merge(a).to_host()
            res["merge"] = (m["start"].tolist(), m["end"].tolist())
            mode = SUBTRACT_LIME if k % 2 == 0 else SUBTRACT_SET
            s = ctx.subtract(a, b, 0, mode).to_host()
            res["sub"] = as_sorted_tuples(s)
            for h in (plan, a, b):
                h.close()
        ctx.close()
        out[k] = (A, B, mode, res)
    except Exception as e:  # surfaced by the main thread
        out[k] = e


def test_concurrent_contexts_match_oracle():
    out = {}
    th = [threading.Thread(target=_job, args=(k, out)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert len(out) == 4
    for k in range(4):
        assert not isinstance(out[k], Exception), out[k]
        A, B, mode, res = out[k]
        assert res["pairs"] == as_sorted_tuples(oracle.intersect(A, B))
        em = oracle.merge(A)
        assert res["merge"] == (em["start"].tolist(), em["end"].tolist())
        assert res["sub"] == as_sorted_tuples(oracle.subtract(A, B, 0, mode))


def test_sets_are_bound_to_their_context():
    sp = Space(NAMES, [1000] * 3)
    c1, c2 = Context(0), Context(0)
    one = (np.array([0], np.int32), np.array([5]), np.array([50]))
    a = c1.set_from_host(sp, *one)
    b = c2.set_from_host(sp, *one)
    for op in (lambda: c1.intersect(a, b), lambda: c1.subtract(a, b), lambda: c2.merge(a),
               lambda: c2.complement(sp, a), lambda: c2.bitset(a)):
        with pytest.raises(LimeError) as ei:
            op()
        assert ei.value.code == 1
    assert c1.intersect(a, c1.set_from_host(sp, *one)).n == 1
    a.close()
    b.close()
    c1.close()
    c2.close()
