"""The C-ABI library on the CPU: it loads, exports every symbol that
include/lime_amd.h declares, and its host-only entry points (contig order,
BED / genome readers, coordinate space, hashing) behave.  No device calls."""
import os
import re

import numpy as np
import pytest

from lime_amd import _ffi
from oracle import oracle
from tests.util import GOLDEN, java_key, read_bed_py, read_genome_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "lime_amd.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lime_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _ffi.load()
    syms = header_symbols()
    assert len(syms) >= 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing
    assert set(syms) == set(_ffi.SIGNATURES), set(syms) ^ set(_ffi.SIGNATURES)
    assert lib.lime_abi_version() == _ffi.ABI_VERSION == 6


def test_no_device_fails_loudly():
    # this container has no GPU: context creation must fail, not fall back
    import ctypes as C
    lib = _ffi.load()
    h = C.c_void_p()
    rc = lib.lime_ctx_create(0, C.byref(h))
    if rc == 0:  # running on a GPU box
        lib.lime_ctx_destroy(h)
        pytest.skip("device present")
    assert rc == 3
    assert b"device" in lib.lime_last_error().lower()


def test_contig_rank_is_java_string_order():
    from lime_amd import java_string_order
    names, _ = read_genome_py(os.path.join(GOLDEN, "genome.txt"))
    rank = java_string_order(names)
    exp = sorted(names, key=java_key)
    assert [names[i] for i in np.argsort(rank)] == exp
    # UTF-16 order differs from UTF-8 byte order for supplementary characters
    r = java_string_order(["\U0001F600", "ﬁ", "chr1", "chr1"])
    assert list(r) == [1, 2, 0, 0]


@pytest.mark.parametrize("name", ["intersect_with_overlap_00.bed", "cpg_20merge.bed", "cpg.bed"])
def test_bed_reader_matches_python(name):
    from lime_amd import read_bed
    path = os.path.join(GOLDEN, name)
    got = read_bed(path)
    chrom, s, e, nm = read_bed_py(path)
    assert got["chrom"] == chrom
    assert (got["start"] == s).all() and (got["end"] == e).all()
    assert got["name"] == nm
    assert (got["strand"] == 0).all()


def test_bed_reader_edge_cases(tmp_path):
    from lime_amd import LimeError, read_bed
    p = tmp_path / "x.bed"
    p.write_text("track name=x\n#c\nbrowser y\n\nchrA\t5\t9\tn1\t0\t+\r\nchrB 1 2\nchrA\t0\t0\t.\t0\t-\n")
    got = read_bed(str(p))
    assert got["chrom"] == ["chrA", "chrB", "chrA"]
    assert list(got["strand"]) == [1, 0, 2]
    assert list(got["end"]) == [9, 2, 0]
    bad = tmp_path / "bad.bed"
    bad.write_text("chr1\tx\t5\n")
    with pytest.raises(LimeError) as ei:
        read_bed(str(bad))
    assert ei.value.code == 6
    with pytest.raises(LimeError):
        read_bed(str(tmp_path / "missing.bed"))


def test_genome_reader_and_space():
    from lime_amd import Space
    sp = Space.from_genome_file(os.path.join(GOLDEN, "genome.txt"))
    names, lens = read_genome_py(os.path.join(GOLDEN, "genome.txt"))
    assert sp.names == sorted(names, key=java_key)
    assert sp.span == sum(lens) + len(lens)
    # off[c+1] = off[c] + len[c] + 1
    assert (np.diff(sp.offsets) == sp.lengths + 1).all()


def test_space_rejects_span_over_2_32():
    from lime_amd import LimeError, Space
    with pytest.raises(LimeError) as ei:
        Space(["a", "b"], [3_000_000_000, 1_500_000_000])
    assert ei.value.code == 2


def test_pair_hash_matches_oracle():
    lib = _ffi.load()
    rng = np.random.default_rng(0)
    for _ in range(100):
        v = [int(x) for x in rng.integers(0, 2**32, 4)]
        assert lib.lime_pair_hash(*v) == oracle.pair_hash(*v)


def test_synth_numpy_is_deterministic_and_in_range():
    from lime_amd import synth
    lens = list(synth.HG38.values())
    c, s, e = synth.uniform(lens, 100000, 0xA, 50, 5000)
    c2, s2, e2 = synth.uniform(lens, 100000, 0xA, 50, 5000)
    assert (c == c2).all() and (s == s2).all()
    L = np.array(lens)[c]
    assert (s >= 0).all() and (e <= L).all()
    w = e - s
    assert w.min() >= 50 and w.max() <= 5000
    # chunked generation == one-shot (counter-based)
    c3, s3, e3 = synth.uniform(lens, 1000, 0xA, 50, 5000, first=500)
    assert (c3 == c[500:1500]).all() and (s3 == s[500:1500]).all()
    # positions ~ uniform: contig frequencies track lengths
    freq = np.bincount(c, minlength=len(lens)) / len(c)
    assert np.abs(freq - np.array(lens) / sum(lens)).max() < 0.01
    pc, ps, pe = synth.pileup(lens, 50000, 0xC, 1000, 150, 150, 600)
    assert (pe - ps).min() >= 150 and (pe <= np.array(lens)[pc]).all()


def test_mulhi_exact():
    from lime_amd import synth
    rng = np.random.default_rng(1)
    x = rng.integers(0, 2**63, 1000, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    m = rng.integers(1, 2**40, 1000, dtype=np.uint64)
    got = synth.mulhi(x, m)
    exp = [(int(a) * int(b)) >> 64 for a, b in zip(x, m)]
    assert [int(v) for v in got] == exp
