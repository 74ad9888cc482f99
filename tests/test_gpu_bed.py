"""Device BED parser (lime_bed_parse_device) against the
engine's host reader (lime_bed_read, bed.cpp) and an independent pure-Python
reader: identical records on the reference's fixture files, on edge-case
text and on a 2e6-line synthetic file; same error codes; and a parsed file
flows into a sorted set without a host round trip."""
import os

import numpy as np
import pytest

from lime_amd import LimeError, Space
from lime_amd.engine import read_bed
from oracle import oracle
from tests.util import GOLDEN, read_bed_py

pytestmark = pytest.mark.gpu

FIXTURES = ["cpg.bed", "cpg_20merge.bed", "intersect_with_overlap_00.bed",
            "intersect_with_overlap_01.bed", "window_with_overlap_01.bed"]


def same_as_host(ctx, text, tmp_path):
    p = tmp_path / "x.bed"
    p.write_bytes(text)
    host = read_bed(str(p))
    d = ctx.parse_bed(text)
    dev = d.to_host()
    assert d.names == host["names"]
    for k in ("contig", "start", "end", "strand"):
        assert (dev[k] == host[k]).all(), k
    assert dev["name"] == host["name"]
    return d, host


@pytest.mark.parametrize("name", FIXTURES)
def test_fixtures_match_host_reader(ctx, name, tmp_path):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        text = f.read()
    d, host = same_as_host(ctx, text, tmp_path)
    chrom, s, e, nm = read_bed_py(os.path.join(GOLDEN, name))
    assert d.n == len(s) and [host["names"][c] for c in host["contig"]] == chrom
    assert (host["start"] == s).all() and (host["end"] == e).all() and host["name"] == nm


def test_edge_cases(ctx, tmp_path):
    text = (b"#comment\ntrack name=x\nbrowser position chr1\n\n"
            b"chr2\t10\t20\tn1\t0\t+\r\n"
            b"chr1\t5\t6\n"
            b"  chrX   7   9   spaced   1   -\n"
            b"chr2\t0\t0\t\t\t?\n"
            b"chr10\t4294967294\t4294967295\tbig\t0\t.\n"
            b"chr1\t1\t2\tlast")  # no trailing newline
    d, host = same_as_host(ctx, text, tmp_path)
    assert d.n == 6
    assert d.names == ["chr2", "chr1", "chrX", "chr10"]
    assert host["strand"].tolist() == [1, 0, 2, 3, 0, 0]
    assert host["name"] == ["n1", "", "spaced", "", "big", "last"]


def test_empty_and_header_only(ctx):
    assert ctx.parse_bed(b"").n == 0
    assert ctx.parse_bed(b"#only a comment\n\n").n == 0


@pytest.mark.parametrize("text,code,line", [
    (b"chr1\t1\t2\nchr1\tx\t5\n", "LIME_ERR_IO", 2),
    (b"chr1\t1\n", "LIME_ERR_IO", 1),
    (b"chr1\t1\t2\nchr1\t3\t4\nchr1\t0\t4294967296\n", "LIME_ERR_RANGE", 3),
    (b"chr1\t-5\t2\n", "LIME_ERR_RANGE", 1),
])
def test_errors(ctx, text, code, line):
    with pytest.raises(LimeError) as ei:
        ctx.parse_bed(text)
    assert code in str(ei.value) and f"line {line}" in str(ei.value)


def test_large_synthetic_matches_host(ctx, tmp_path):
    rng = np.random.default_rng(3)
    n = 2_000_000
    names = [f"chr{i}" for i in range(1, 23)] + ["chrX", "chrY", "chrM", "chrUn_KI270302v1"]
    c = rng.integers(0, len(names), n)
    s = rng.integers(0, 250_000_000, n)
    e = s + rng.integers(0, 5000, n)
    st = rng.choice(np.array(["+", "-", "."]), n)
    lines = [f"{names[a]}\t{b}\t{x}\tr{i}\t0\t{y}" for i, (a, b, x, y) in
             enumerate(zip(c.tolist(), s.tolist(), e.tolist(), st.tolist()))]
    text = ("\n".join(lines) + "\n").encode()
    d, host = same_as_host(ctx, text, tmp_path)
    assert d.n == n


def test_parsed_file_builds_set(ctx):
    # device parse -> device remap -> sorted set: same merge as the host path
    with open(os.path.join(GOLDEN, "cpg.bed"), "rb") as f:
        text = f.read()
    d = ctx.parse_bed(text)
    chrom, s, e, _ = read_bed_py(os.path.join(GOLDEN, "cpg.bed"))
    ext = {}
    for cname, x in zip(chrom, e):
        ext[cname] = max(ext.get(cname, 0), int(x))
    sp = Space(list(ext), list(ext.values()))
    A = d.to_set(sp)
    got = ctx.merge(A).to_host()
    ids = np.array([sp.index[x] for x in chrom], np.int32)
    exp = oracle.merge((ids, s, e))
    assert got["start"].tolist() == exp["start"].tolist()
    assert got["end"].tolist() == exp["end"].tolist()
    assert got["contig"].tolist() == exp["contig"].tolist()


def _bed3(contig, start, end, names):
    return "".join(f"{names[c]}\t{s}\t{e}\n" for c, s, e in zip(contig, start, end)).encode()


def test_writer_set_and_results(ctx):
    # device BED writer: sorted set rows, merge runs and complement gaps, as
    # BED3 text equal to the host formatting of the same arrays
    rng = np.random.default_rng(12)
    names = ["chr1", "chr10", "chr2", "chrX"]
    lens = [300000, 200000, 250000, 100000]
    sp = Space(names, lens)
    n = 50000
    c = rng.integers(0, 4, n).astype(np.int32)
    s = rng.integers(0, 90000, n).astype(np.int64)
    e = s + rng.integers(0, 3000, n)
    A = ctx.set_from_host(sp, c, s, e)
    h = A.to_host()
    assert A.to_bed() == _bed3(h["contig"], h["start"], h["end"], sp.names)
    m = ctx.merge(A)
    hm = m.to_host()
    assert m.to_bed() == _bed3(hm["contig"], hm["start"], hm["end"], sp.names)
    comp = ctx.complement(sp, A)
    hc = comp.to_host()
    assert comp.to_bed() == _bed3(hc["contig"], hc["start"], hc["end"], sp.names)
    # round trip: writer -> device parser -> same rows
    d = ctx.parse_bed(m.to_bed()).to_host()
    assert d["start"].tolist() == hm["start"].tolist() and d["end"].tolist() == hm["end"].tolist()


def test_writer_large_lines_and_empty(ctx):
    # long contig names push a 256-row block past the LDS text buffer (the
    # direct-store fallback); an empty set formats to b""
    long = "contig_" + "x" * 200
    sp = Space([long, "c2"], [10**9, 5000])
    n = 3000
    c = np.full(n, sp.index[long], np.int32)
    s = np.arange(n, dtype=np.int64) * 1000 + 999_000_000 - 3_000_000
    e = s + 7
    A = ctx.set_from_host(sp, c, s, e)
    h = A.to_host()
    assert A.to_bed() == _bed3(h["contig"], h["start"], h["end"], sp.names)
    E = ctx.set_from_host(sp, np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, np.int64))
    assert E.to_bed() == b""
