"""bin/lime-submit: the command surface of bin/lime-submit + LimeMain
(LimeMain.scala:30-57), backed by the C++ operator mirror (include/lime_amd.hpp)."""
import os
import subprocess

import pytest

from tests.util import GOLDEN, expected

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "lime-submit")


def run(*args):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=120)


def g(name):
    return os.path.join(GOLDEN, name)


def test_usage_and_version():
    r = run()
    assert r.returncode == 0 and "Choose one of the following commands" in r.stdout
    for cmd in ("complement", "intersect", "merge", "subtract", "sort", "window", "cluster",
                "closest"):
        assert cmd in r.stdout
    r = run("-version")
    assert r.returncode == 0 and r.stdout.startswith("Version 0")
    # spark args before "--" are accepted and ignored (bin/lime-submit:7-23)
    r = run("--master", "local[4]", "--", "-version")
    assert r.returncode == 0 and "Version 0" in r.stdout
    r = run("nonsense")
    assert "Choose one of the following commands" in r.stdout


def test_no_device_fails_loudly():
    r = run("intersect", g("intersect_with_overlap_00.bed"), g("intersect_with_overlap_01.bed"))
    if r.returncode == 0:
        pytest.skip("device present")
    assert r.returncode == 1 and "status 3" in r.stderr


def lines(r):
    assert r.returncode == 0, r.stderr
    return [l.split("\t") for l in r.stdout.strip().split("\n") if l]


@pytest.mark.gpu
def test_cli_intersect_subtract_merge_complement_sort():
    ex = expected()
    out = lines(run("--", "intersect", g("intersect_with_overlap_00.bed"),
                    g("intersect_with_overlap_01.bed")))
    assert [[c, int(s), int(e)] for c, s, e, *_ in out] == ex["intersection_full"]
    assert out[0][3:] == ["CpG:_30", "CpG:_116"]
    out = lines(run("subtract", g("intersect_with_overlap_00.bed"),
                    g("intersect_with_overlap_01.bed")))
    assert [[c, int(s), int(e)] for c, s, e, *_ in out] == ex["subtract"]
    out = lines(run("merge", g("cpg_20merge.bed")))
    assert out == [["chr1", "28735", "30000", "20"]]
    out = lines(run("complement", g("cpg_20merge.bed"), g("genome.txt")))
    assert [[c, int(s), int(e)] for c, s, e in out] == ex["complement"]
    out = lines(run("sort", g("cpg.bed")))
    assert len(out) == 28691
    key = [(c.encode("utf-16-be"), int(s), int(e)) for c, s, e, _ in out]
    assert key == sorted(key)


@pytest.mark.gpu
def test_cli_window():
    # WindowSuite.scala:8-34 through the CLI (cli/Window.scala, distance 1000)
    out = lines(run("window", g("intersect_with_overlap_00.bed"), g("window_with_overlap_01.bed")))
    assert [[[c, int(s), int(e)]] for c, s, e, *_ in out] == \
        [[p[0]] for p in expected()["window"]]
    # -distance 9 keeps the 9-base gap (distance 10 > 9 drops it: gap + 1)
    out = lines(run("window", g("intersect_with_overlap_00.bed"), g("window_with_overlap_01.bed"),
                    "-distance", "10"))
    assert ["chr1", "135453", "139441", "CpG:_99", "CpG:_116"] in out
    out = lines(run("window", g("intersect_with_overlap_00.bed"), g("window_with_overlap_01.bed"),
                    "-distance", "9"))
    assert ["chr1", "135453", "139441", "CpG:_99", "CpG:_116"] not in out


@pytest.mark.gpu
def test_cli_cluster():
    # cli/Cluster.scala + ClusterSuite: one cluster keyed by the first member
    out = lines(run("cluster", g("cpg_20merge.bed")))
    assert len(out) == 1 and out[0][3] == "20"
    assert out[0][:3] == ["chr1", "28735", "29810"]


@pytest.mark.gpu
def test_cli_closest():
    # ClosestSuite.scala:8-49 through the CLI (cli/Closest.scala: SingleClosest
    # on stranded keys; the fixtures carry no strand): all 24 pairs in order
    out = lines(run("closest", g("intersect_with_overlap_00.bed"),
                    g("intersect_with_overlap_01.bed")))
    right = {n: [c, int(s), int(e)] for c, s, e, n in
             (ln.rstrip("\n").split("\t")[:4] for ln in open(g("intersect_with_overlap_01.bed")))}
    got = [[[c, int(s), int(e)], right[r]] for c, s, e, _, r in out]
    assert got == [list(map(list, p)) for p in expected()["closest"]]


@pytest.mark.gpu
def test_cli_genome_cut_into_spaces(tmp_path):
    # a genome past 2^32 bases is cut into consecutive spaces (u32 engine
    # coordinates); LIME_SPAN_CAP cuts hg19 (C1's inputs) into ~6 the same
    # way: every command prints exactly its one-space output
    from tests.test_gpu_configs import c1_inputs
    _, _, (pa, pb), (gn, gl) = c1_inputs(tmp_path)
    gfile = tmp_path / "genome.txt"
    gfile.write_text("".join(f"{n}\t{ln}\n" for n, ln in zip(gn, gl)))
    cmds = [("intersect", pa, pb), ("subtract", pa, pb), ("merge", pa),
            ("complement", pa, str(gfile)), ("sort", pa), ("window", pa, pb),
            ("cluster", pa), ("closest", pa, pb)]
    env = dict(os.environ)
    env.pop("LIME_SPAN_CAP", None)
    one = [subprocess.run([CLI, *c], capture_output=True, text=True, timeout=300, env=env)
           for c in cmds]
    env["LIME_SPAN_CAP"] = "600000000"
    cut = [subprocess.run([CLI, *c], capture_output=True, text=True, timeout=300, env=env)
           for c in cmds]
    for c, x, y in zip(cmds, one, cut):
        assert x.returncode == 0 and y.returncode == 0, (c[0], x.stderr, y.stderr)
        assert x.stdout and x.stdout == y.stdout, c[0]
