"""the RCCL exchange runs on hardware.  A one-rank RCCL
process group with LMI_FORCE_EXCHANGE=1 takes every step form's G > 1 branch
(Searcher.search / lists, GraphedSearch captured and pipelined, the
StreamedSearch graphs F1 + F2 with the captured all-gather), bitwise equal to
the plain one-GPU path in both arithmetics (tests/rccl_worker.py, its own
process: the pytest process keeps no process group)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(300)
def test_one_rank_rccl_exchange_equals_the_one_gpu_path():
    env = dict(os.environ, LMI_FORCE_EXCHANGE="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               LMI_DIST_TIMEOUT_S="120")
    env.pop("MASTER_PORT", None)
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py")], env=env,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "RCCL forced exchange OK" in p.stdout
