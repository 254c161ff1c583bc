"""Direct xGMI collectives (csrc/kernels/xgmi.hip, mihvd/parallel/xgmi.py) against plain fp32 /
gloo references, eager and replayed from a HIP graph, plus the failure path (a peer past the
device-side timeout). Two ranks share the box's one GPU: the IPC mapping, the cross-process phase
barriers and the data movement are the code an 8-GPU node runs over xGMI (cross-GPU coherence
itself is only exercised on a multi-GPU node; see docs/ARCHITECTURE.md)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "workers", "xgmi_worker.py")


def _run(tmp_path, scenario, port, extra_env=None):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), WORKER, scenario, str(tmp_path)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return [json.loads((tmp_path / f"{scenario}.{r}.json").read_text()) for r in range(2)]


def test_xgmi_oneshot_allreduce_two_ranks(tmp_path):
    for o in _run(tmp_path, "allreduce", 29541):
        for e in o["eager"]:
            assert e["max_err"] <= 1e-6 * max(1.0, e["n"] ** 0.5), e
        for g in o["graph"]:
            assert g["max_err"] == 0.0, g


def test_xgmi_region_gather_and_reduce_two_ranks(tmp_path):
    for o in _run(tmp_path, "region", 29542):
        assert len(o["checks"]) == 7
        for c in o["checks"]:
            assert c["rows_ok"], c
            # the kernel sums in rank order exactly like the reference loop
            assert c["sum_bitwise"], c


def test_xgmi_peer_timeout_poisons_and_raises(tmp_path):
    r0, r1 = _run(tmp_path, "timeout", 29543, {"MIHVD_XGMI_TIMEOUT_MS": "300"})
    assert r0["first_nan"] and r0["raised"], r0
    assert "rank(s) [1]" in r0["msg"], r0
    assert r0["first_s"] < 2.5, r0           # bounded by the timeout, not by the late peer
    assert r0["second_nan"] and r0["second_s"] < 1.0, r0  # poisoned: no second wait
    assert not r1["first_nan"] and not r1["raised"], r1   # the late rank found its peer's signal
    # the timeout reached the host-coherent mirror the health monitor watches (bit 1 + poison)
    assert r0["mirror"] == 0x80000002, r0
    assert r0["monitor"][0] == 6 and "xgmi test" in r0["monitor"][1], r0
    assert r1["mirror"] == 0 and r1["monitor"] == [0, ""], r1
