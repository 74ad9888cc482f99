"""One context on two streams (lime_ctx_set_stream): the pool hands a block
released on one stream to work on the other only after the releasing work is
done (events), so sets sorted on one stream and joined on another, batch
after batch, keep giving the oracle's results."""
import numpy as np
import pytest

from oracle import oracle
from tests.util import as_sorted_tuples, random_sets

pytestmark = pytest.mark.gpu


def test_two_streams_batches(ctx):
    import torch

    from lime_amd import Space
    sp = Space(["chr1", "chr2", "chr3"], [60000] * 3)
    side, main = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        for seed in range(6):
            rng = np.random.default_rng(100 + seed)
            A, B = random_sets(rng, 20000, 15000, n_contigs=3, contig_len=60000, max_len=400,
                               zero_frac=0.05, dup_frac=0.05, book_frac=0.05)
            ctx.set_stream(side.cuda_stream)
            a, b = ctx.set_from_host(sp, *A), ctx.set_from_host(sp, *B)
            done = torch.cuda.Event()
            done.record(side)
            ctx.set_stream(main.cuda_stream)
            main.wait_event(done)
            plan = ctx.intersect(a, b)
            m = ctx.merge(a)
            exp = oracle.intersect(A, B)
            p = plan.fill_host()
            got = {"contig": A[0][p["a_row"]], "start": p["start"], "end": p["end"],
                   "a_row": p["a_row"], "b_row": p["b_row"]}
            assert as_sorted_tuples(got) == as_sorted_tuples(exp)
            assert m.to_host()["start"].tolist() == oracle.merge(A)["start"].tolist()
            for h in (plan, m, a, b):
                h.close()
    finally:
        ctx.set_stream(None)
