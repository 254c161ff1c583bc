"""Direct xGMI one-shot allreduce (csrc/kernels/xgmi.hip, mihvd/parallel/xgmi.py) against a plain
fp32 sum, eager and replayed from a HIP graph. Two ranks share the box's one GPU: the IPC mapping,
the cross-process device barrier and the double-buffered slots are the same code the 8-GPU node
runs over xGMI."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "workers", "xgmi_worker.py")


def test_xgmi_oneshot_allreduce_two_ranks(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29541", WORKER, str(tmp_path)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    for r in range(2):
        o = json.loads((tmp_path / f"xgmi.{r}.json").read_text())
        for e in o["eager"]:
            assert e["max_err"] <= 1e-6 * max(1.0, e["n"] ** 0.5), e
        for g in o["graph"]:
            assert g["max_err"] == 0.0, g
