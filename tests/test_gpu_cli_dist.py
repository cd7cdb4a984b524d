"""The reference's own interface sharded over G processes:
`search.py --gpus G` (li.dist.launch_ranks starts the ranks; LearnedIndex's
process-group mode builds one stripe of every bucket per rank) writes the same
eval H5 files, byte for byte in `knns` and `dists`, as one process -- through
`LearnedIndex.search` (-bp 25: R = 4 of 16 buckets) and
`LearnedIndex.search_single` (-bp 7: R = 1), search.py:115-164.

The ranks share the box's one GPU over gloo (LMI_DIST_BACKEND=gloo: RCCL
refuses two ranks on one device); the 8-GPU node runs the same code over RCCL.
Every run after the first loads the router the first one pickled (--save, then
--index), so all runs index the same buckets."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

from li import h5

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd", "search.py")
ARGS = ["--synthetic", "20000", "--size", "100K", "--n-categories", "16", "--epochs", "3",
        "--model-type", "MLP", "--lr", "0.01", "-bp", "7", "25"]


def _cli(cwd, extra, timeout=240, **env_extra):
    os.makedirs(cwd, exist_ok=True)
    env = dict(os.environ, LMI_DIST_BACKEND="gloo", LMI_DIST_TIMEOUT_S="120", **env_extra)
    env.pop("WORLD_SIZE", None)
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, CLI] + ARGS + list(extra), cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    # (progress for a long run: each CLI run is one build or load + 2 searches)
    print(f"search.py {' '.join(extra)}: {time.time() - t0:.1f} s", flush=True)
    return r


def _results(cwd):
    out = {}
    for f in sorted(glob.glob(os.path.join(cwd, "result", "pca96v2", "100K", "*.h5"))):
        b = "buck=4" if "buck=4" in f else "buck=1"
        out[b] = (h5.read_dataset(f, "knns"), h5.read_dataset(f, "dists"))
    assert set(out) == {"buck=1", "buck=4"}, out.keys()
    return out


@pytest.mark.timeout(900)
def test_cli_gpus_writes_the_one_process_results(tmp_path):
    built = str(tmp_path / "built")
    _cli(built, ["--save", "True"])
    pkl = glob.glob(os.path.join(built, "models", "*.pkl"))
    assert len(pkl) == 1
    one = str(tmp_path / "one")
    _cli(one, ["--index", pkl[0]])
    ref = _results(one)
    # the loaded router labels the corpus as the build did: same answers
    for b, (kn, di) in _results(built).items():
        np.testing.assert_array_equal(kn, ref[b][0])
        np.testing.assert_array_equal(di, ref[b][1])
    # the reference's flow without search.py's attach: the first call attaches
    # (LMI_AUTO_ATTACH=1) instead of every call hashing the corpus
    auto = str(tmp_path / "auto")
    _cli(auto, ["--index", pkl[0]], LMI_NO_ATTACH="1", LMI_AUTO_ATTACH="1")
    for b, (kn, di) in _results(auto).items():
        np.testing.assert_array_equal(kn, ref[b][0])
        np.testing.assert_array_equal(di, ref[b][1])
    for G in (2, 3):
        cwd = str(tmp_path / f"g{G}")
        _cli(cwd, ["--index", pkl[0], "--gpus", str(G)])
        got = _results(cwd)
        for b in ("buck=1", "buck=4"):
            assert got[b][0].dtype == np.uint32 and got[b][1].dtype == np.float64
            np.testing.assert_array_equal(got[b][0], ref[b][0], err_msg=f"G={G} {b} knns")
            np.testing.assert_array_equal(got[b][1], ref[b][1], err_msg=f"G={G} {b} dists")
        # only rank 0 wrote (one file per bucket count, no partial writers)
        assert len(glob.glob(os.path.join(cwd, "result", "pca96v2", "100K", "*.h5"))) == 2


@pytest.mark.timeout(600)
def test_cli_gpus_builds_on_rank0_and_shares_the_router(tmp_path):
    """Without --index: rank 0 trains, the router and labels are broadcast,
    every rank indexes the same buckets (the answers are complete and sorted;
    the one-process build is a separate training run, compared only when
    torch's GPU training reproduced itself bit for bit)."""
    cwd = str(tmp_path / "g2")
    r = _cli(cwd, ["--gpus", "2", "--save", "True"])
    got = _results(cwd)
    kn, di = got["buck=4"]
    assert kn.shape == (10_000, 10) and np.all(kn > 0)
    assert np.all(np.diff(di, axis=1) >= 0)
    assert len(glob.glob(os.path.join(cwd, "models", "*.pkl"))) == 1   # rank 0 only
    assert "Searching with 4 buckets" in r.stderr
