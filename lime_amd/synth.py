"""Synthetic interval sets -- numpy restatement of
lime_amd/csrc/synth.hip, bit-identical to the device generator so the CPU
oracle, the GPU path and every shard count see the same rows.

    rng(seed, i, k) = mix64(seed * 0x9E3779B97F4A7C15 + 8 i + k)  (mod 2^64)
    mulhi(x, m)     = floor(x * m / 2^64)
"""
import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
M32 = np.uint64(0xFFFFFFFF)

# hg38 primary assembly (UCSC hg38.chrom.sizes), SURVEY.md 8(d)
HG38 = {
    "chr1": 248956422, "chr2": 242193529, "chr3": 198295559, "chr4": 190214555,
    "chr5": 181538259, "chr6": 170805979, "chr7": 159345973, "chr8": 145138636,
    "chr9": 138394717, "chr10": 133797422, "chr11": 135086622, "chr12": 133275309,
    "chr13": 114364328, "chr14": 107043718, "chr15": 101991189, "chr16": 90338345,
    "chr17": 83257441, "chr18": 80373285, "chr19": 58617616, "chr20": 64444167,
    "chr21": 46709983, "chr22": 50818468, "chrX": 156040895, "chrY": 57227415,
    "chrM": 16569,
}


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rng(seed, i, k):
    i = np.asarray(i, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(np.uint64(seed) * GOLD + i * np.uint64(8) + np.uint64(k))


def mulhi(x, m):
    x = np.asarray(x, dtype=np.uint64)
    m = np.asarray(m, dtype=np.uint64)
    xh, xl = x >> np.uint64(32), x & M32
    mh, ml = m >> np.uint64(32), m & M32
    with np.errstate(over="ignore"):
        hl = xh * ml
        lh = xl * mh
        ll = xl * ml
        carry = ((hl & M32) + (lh & M32) + (ll >> np.uint64(32))) >> np.uint64(32)
        return xh * mh + (hl >> np.uint64(32)) + (lh >> np.uint64(32)) + carry


def _place(pos, l, lengths):
    base = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint64)
    c = np.searchsorted(base[:-1], pos, side="right").astype(np.int64) - 1
    L = np.asarray(lengths, dtype=np.uint64)[c]
    l = np.minimum(l, L)
    local = np.minimum(pos - base[c], L - l)
    return c.astype(np.int32), local.astype(np.int64), (local + l).astype(np.int64)


def uniform(lengths, n, seed, len_lo, len_hi, first=0):
    """Rows [first, first+n): contig index (into `lengths`), start, end."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    G = np.uint64(int(lengths.sum()))
    i = np.arange(first, first + n, dtype=np.uint64)
    pos = mulhi(rng(seed, i, 0), G)
    l = np.uint64(len_lo) + mulhi(rng(seed, i, 1), np.uint64(len_hi - len_lo + 1))
    return _place(pos, l, lengths)


def pileup(lengths, n, seed, n_centres, sigma, len_lo, len_hi, first=0):
    """ChIP-seq-like pile-ups: Irwin-Hall N(0, sigma) offsets around K centres."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    G = int(lengths.sum())
    s1 = seed + 1
    i = np.arange(first, first + n, dtype=np.uint64)
    k = mulhi(rng(s1, i, 0), np.uint64(n_centres))
    cpos = mulhi(rng(seed, k, 0), np.uint64(G)).astype(np.int64)
    total = np.zeros(n, dtype=np.int64)
    for q in (1, 2, 3):
        x = rng(s1, i, q)
        for h in range(4):
            total += ((x >> np.uint64(16 * h)) & np.uint64(0xFFFF)).astype(np.int64)
    off = ((total - 393210) * int(sigma)) >> 16
    p = np.clip(cpos + off, 0, G - 1).astype(np.uint64)
    l = np.uint64(len_lo) + mulhi(rng(s1, i, 4), np.uint64(len_hi - len_lo + 1))
    return _place(p, l, lengths)
