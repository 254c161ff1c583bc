"""Distributed paths of the fused trainer on one MI355X (the multi-GPU node is the driver's):
RCCL allreduce captured inside the HIP graph, and data-parallel equivalence across two ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "workers", "fused_worker.py")


def _gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_rccl_allreduce_inside_hip_graph(tmp_path):
    _gpu()
    env = dict(os.environ, MIHVD_FORCE_COLLECTIVES="1", PYTHONPATH=ROOT, MIHVD_BACKEND="nccl")
    for k in ("RANK", "WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, WORKER, "rccl_graph", str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads((tmp_path / "rccl_graph.json").read_text())
    assert r["captured"], "RCCL allreduce could not be captured into the HIP graph"
    assert r["steps"] == 22 and r["bitwise"], r


@pytest.mark.parametrize("gather", ["1", "0"])
def test_fused_data_parallel_equivalence_two_ranks(tmp_path, gather):
    """gather=1: dW3 from all-gathered factors (the default data plane); gather=0: bucket allreduce."""
    _gpu()
    env = dict(os.environ, MIHVD_BACKEND="gloo", PYTHONPATH=ROOT, MIHVD_FC_GATHER=gather)
    cmd = [sys.executable, "-m", "mihvd.runner", "-np", "2", sys.executable, WORKER, "dp_gloo", str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    for r in range(2):
        o = json.loads((tmp_path / f"dp_gloo.{r}.json").read_text())
        assert o["rank_spread"] == 0.0
        assert o["grad_rel"] < 1e-4, o
        assert o["rel_update_diff"] < 0.05, o
