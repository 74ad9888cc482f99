"""bench.py's own rank launcher (`bench.py --gpus N` with no external
launcher): N fresh children with the rendezvous environment, rank 0's line
relayed, a failing rank stops the job, and a WORLD_SIZE that disagrees with
--gpus is refused.  CPU only: the child here is a stand-in script that reads
the environment the way bench.py's main() does."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import json, os, sys
import torch.distributed as dist
w, r = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
if "--fail" in sys.argv and r == w - 1:
    sys.exit(7)
dist.init_process_group("gloo")
import torch
t = torch.tensor([r + 1])
dist.all_reduce(t)
if r == 0:
    print(json.dumps({"n_gpus": w if "--lie" not in sys.argv else 1, "sum": int(t)}),
          flush=True)
dist.destroy_process_group()
'''


@pytest.fixture()
def child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def _spawn(child, n, argv):
    code = ("import sys, bench; sys.exit(bench.spawn_ranks(%d, script=%r, argv=%r))"
            % (n, child, argv))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_ranks_rendezvous(child, n):
    r = _spawn(child, n, [])
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec == {"n_gpus": n, "sum": n * (n + 1) // 2}


def test_spawn_ranks_failing_rank(child):
    r = _spawn(child, 2, ["--fail"])
    assert r.returncode == 7


def test_spawn_ranks_wrong_world_reported(child):
    r = _spawn(child, 2, ["--lie"])
    assert r.returncode != 0 and "n_gpus" in r.stderr


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
