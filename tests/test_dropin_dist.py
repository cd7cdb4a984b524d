"""Host logic of LearnedIndex's process-group mode, over
gloo on the CPU (no HIP device): rank 0's trained router and object labels
reach every rank (`_share_build`), only rank 0 writes result and model files,
and the mode is entered from a launcher's environment.  The GPU side --
search.py --gpus G writing the one-process H5 files -- is
tests/test_gpu_cli_dist.py."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from li.LearnedIndex import LearnedIndex
    from li.model import NeuralNetwork
    from li.utils import save_as_pickle
    li = LearnedIndex()
    pg = li._proc_group()                 # entered from WORLD_SIZE > 1
    assert pg is not None and pg[1] == rank and pg[2] == world
    assert pg[3] is None  # (the stripe's chunk: by the index's size, li.index.default_chunk_rows)
    built = None
    if rank == 0:
        torch.manual_seed(7)
        nn = NeuralNetwork(input_dim=96, output_dim=16, lr=0.01, model_type="MLP-5")
        labels = np.random.default_rng(3).integers(0, 16, 1000)
        li.model = nn
        built = (nn, labels)
    labels = li._share_build(pg, built, 96, 16, 0.01, "MLP-5")
    state = {k: v.detach().cpu() for k, v in li.model.model.state_dict().items()}
    torch.save({"labels": torch.from_numpy(np.asarray(labels)), "state": state},
               os.path.join(out_dir, f"rank{rank}.pt"))
    save_as_pickle(os.path.join(out_dir, "model.pkl") if rank == 0 else
                   os.path.join(out_dir, f"model{rank}.pkl"), li)
    dist.barrier()
    dist.destroy_process_group()


def test_build_is_shared_from_rank0_and_only_rank0_writes(tmp_path):
    world = 3
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for g in got[1:]:
        assert torch.equal(g["labels"], got[0]["labels"])
        assert g["state"].keys() == got[0]["state"].keys()
        for k in g["state"]:
            assert torch.equal(g["state"][k], got[0]["state"][k])
    assert (tmp_path / "model.pkl").exists()
    assert not any((tmp_path / f"model{r}.pkl").exists() for r in range(1, world))
    # the pickle holds the reference's attributes, not the process group
    from li.index_io import load_index
    li = load_index(str(tmp_path / "model.pkl"))
    assert li._pg is None and li.model is not None


def test_no_process_group_mode_without_a_launcher(monkeypatch):
    from li.LearnedIndex import LearnedIndex
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert LearnedIndex()._proc_group() is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LMI_SHARD", "0")
    assert LearnedIndex()._proc_group() is None


def test_gpus_arg():
    from li.dist import gpus_arg
    assert gpus_arg(["--size", "10M", "--gpus", "8"]) == 8
    assert gpus_arg(["--gpus=2"]) == 2
    assert gpus_arg(["-bp", "4"]) == 1


def _slow_build_worker(rank, world, port, out_dir):
    """Rank 0 builds for longer than the process group's timeout (3 s here):
    the other ranks wait on the store (LearnedIndex._build_done), so the
    broadcast after it does not time out; a second build that
    fails on rank 0 raises on every rank."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LMI_DIST_TIMEOUT_S="3")
    from li.LearnedIndex import LearnedIndex
    from li.model import NeuralNetwork
    li = LearnedIndex()
    pg = li._proc_group()
    built = None
    if rank == 0:
        time.sleep(6.0)
        torch.manual_seed(7)
        li.model = NeuralNetwork(input_dim=96, output_dim=16, lr=0.01, model_type="MLP")
        built = (li.model, np.arange(50) % 16)
    li._build_done(pg, None)
    labels = li._share_build(pg, built, 96, 16, 0.01, "MLP")
    failed = ""
    try:
        if rank == 0:
            li._build_done(pg, "ValueError('boom')")
        else:
            li._build_done(pg, None)
    except RuntimeError as e:
        failed = str(e)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{int(np.asarray(labels).sum())}|{failed}")
    dist.barrier()
    dist.destroy_process_group()


def test_slow_rank0_build_does_not_time_out_the_other_ranks(tmp_path):
    world = 3
    mp.spawn(_slow_build_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [(tmp_path / f"r{r}.txt").read_text().split("|") for r in range(world)]
    assert all(g[0] == got[0][0] for g in got)
    assert got[0][1] == ""
    assert all("boom" in g[1] for g in got[1:])
