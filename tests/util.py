"""Test helpers: an independent pure-Python BED reader (so the oracle's
inputs do not depend on the product's parser), Java String ordering, and
sorted-list comparison of outputs."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def java_key(s):
    return s.encode("utf-16-be")


def read_bed_py(path):
    chrom, start, end, name = [], [], [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\r\n")
            if not line or line.startswith(("#", "track", "browser")):
                continue
            p = line.split("\t")
            chrom.append(p[0])
            start.append(int(p[1]))
            end.append(int(p[2]))
            name.append(p[3] if len(p) > 3 else "")
    return chrom, np.array(start, np.int64), np.array(end, np.int64), name


def read_genome_py(path):
    names, lens = [], []
    with open(path) as f:
        for line in f:
            p = line.rstrip("\r\n").split("\t")
            if len(p) >= 2:
                names.append(p[0])
                lens.append(int(p[1]))
    return names, lens


def ranked(names_all):
    """name -> rank in Java String order."""
    uniq = sorted(set(names_all), key=java_key)
    return {n: i for i, n in enumerate(uniq)}


def expected():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)


def as_sorted_tuples(res, keys=("contig", "start", "end", "a_row", "b_row")):
    cols = [np.asarray(res[k]).astype(np.int64) for k in keys if k in res]
    if not cols or len(cols[0]) == 0:
        return []
    arr = np.stack(cols, axis=1)
    order = np.lexsort(arr.T[::-1])
    return [tuple(r) for r in arr[order].tolist()]


def random_sets(rng, n_a, n_b, n_contigs=3, contig_len=20000, max_len=300, zero_frac=0.0,
                dup_frac=0.0, book_frac=0.0):
    """Seeded small interval sets with the edge cases the reference tests skip:
    zero-width rows, exact duplicates and book-ended neighbours."""
    def one(n):
        c = rng.integers(0, n_contigs, n).astype(np.int32)
        s = rng.integers(0, contig_len - max_len, n).astype(np.int64)
        l = rng.integers(1, max_len, n).astype(np.int64)
        if zero_frac:
            l[rng.random(n) < zero_frac] = 0
        e = s + l
        if dup_frac and n > 1:
            k = rng.random(n) < dup_frac
            src = rng.integers(0, n, n)
            c[k], s[k], e[k] = c[src[k]], s[src[k]], e[src[k]]
        if book_frac and n > 1:
            k = np.nonzero(rng.random(n) < book_frac)[0]
            src = rng.integers(0, n, len(k))
            c[k] = c[src]
            s[k] = e[src]
            e[k] = np.minimum(s[k] + rng.integers(0, max_len, len(k)), contig_len)
        return c, s, e
    return one(n_a), one(n_b)
