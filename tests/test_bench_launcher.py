"""bench.py --gpus N without torchrun starts N rank processes itself
(bench.launch_ranks): RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* reach every rank,
rank 0's single JSON line is relayed, and a failing rank fails the launch
(the other ranks are stopped rather than left waiting at a collective).
Driven here with a stand-in rank script on gloo (no GPU)."""
import json
import os
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    import torch, torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    if "--fail" in sys.argv and rank == 1:
        sys.exit(3)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0 and "--big" in sys.argv:
        print("x" * 300000)   # more than a pipe buffer, before the collective
    dist.barrier()
    if rank == 0:
        print(json.dumps({"n_gpus": world, "max": float(t), "local": os.environ["LOCAL_RANK"]}))
    dist.barrier()
    dist.destroy_process_group()
""")


@pytest.fixture
def script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launcher_runs_n_ranks_and_relays_rank0(script, capfd, monkeypatch):
    import bench
    monkeypatch.setenv("LMI_DIST_BACKEND", "gloo")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench._gpus_arg(["--steps", "3", "--gpus", "2"]) == 2
    assert bench._gpus_arg(["--gpus=4"]) == 4
    rc = bench.launch_ranks(2, [], script=script)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    line = json.loads(out[-1])
    assert line["n_gpus"] == 2 and line["max"] == 2.0 and line["local"] == "0"


def test_launcher_fails_when_a_rank_fails(script, monkeypatch):
    import bench
    monkeypatch.setenv("LMI_DIST_BACKEND", "gloo")
    rc = bench.launch_ranks(2, ["--fail"], script=script)
    assert rc == 3


def test_launcher_relays_more_than_a_pipe_buffer(script, capfd, monkeypatch):
    """Rank 0 writes 300 KB to stdout before a collective: the relay does not
    block it (an unread pipe would, leaving the other rank at the barrier)."""
    import bench
    monkeypatch.setenv("LMI_DIST_BACKEND", "gloo")
    monkeypatch.setenv("LMI_DIST_TIMEOUT_S", "60")
    rc = bench.launch_ranks(2, ["--big"], script=script)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out[-2]) == 300000
    assert json.loads(out[-1])["n_gpus"] == 2
