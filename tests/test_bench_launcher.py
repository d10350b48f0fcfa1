"""bench.py's own multi-rank launcher (``python bench.py --gpus N`` without torchrun), on CPU with gloo.

The driver may start the scaling bench as ``python bench.py --gpus N``; the launcher must then run N rank
processes with torchrun's environment, and every rank must refuse a world that is not one rank per ``--gpus``.
"""

import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_rank_envs_are_torchrun_like():
    envs = bench.rank_envs(4, 29511, base={"KEEP": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["KEEP"] == "1"


CHILD = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    assert r == int(os.environ["LOCAL_RANK"])
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    ranks = [None] * w
    dist.all_gather_object(ranks, r)
    if r == 0:
        print(json.dumps({"world": w, "sum": t.item(), "ranks": ranks}))
    if os.environ.get("FAIL_RANK") == str(r):
        sys.exit(3)
    dist.destroy_process_group()
""")


def test_launch_ranks_runs_a_gloo_world(tmp_path):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        rc = bench.launch_ranks(3, [sys.executable, str(child)], stdout=f)
    assert rc == 0
    lines = out.read_text().strip().splitlines()
    assert not any(ln.startswith("[Gloo] Rank 1") for ln in lines)  # only rank 0 writes stdout
    line = json.loads(lines[-1])
    assert line == {"world": 3, "sum": 6.0, "ranks": [0, 1, 2]}


def test_launch_ranks_reports_a_failing_rank(tmp_path, monkeypatch):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    monkeypatch.setenv("FAIL_RANK", "1")
    with open(tmp_path / "out.txt", "w") as f:
        rc = bench.launch_ranks(2, [sys.executable, str(child)], stdout=f)
    assert rc == 3


def test_rank_refuses_a_world_other_than_gpus():
    """A rank started with WORLD_SIZE != --gpus exits before it touches the GPU."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr
