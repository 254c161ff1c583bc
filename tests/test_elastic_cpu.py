"""Elastic training (mihvd.elastic + mihvdrun --min-np): multi-process gloo jobs on the CPU."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "workers", "elastic_worker.py")

pytestmark = pytest.mark.slow


def run(tmp_path, scenario, launcher_args):
    env = dict(os.environ, MIHVD_BACKEND="gloo", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               MIHVD_ELASTIC_GRACE_SECONDS="20")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "mihvd.runner", *launcher_args, sys.executable, WORKER, scenario, str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    outs = [json.loads(open(f).read()) for f in sorted(glob.glob(str(tmp_path / f"{scenario}.w*.json")))]
    return p, outs


def _consistent(outs):
    ref = outs[0]["allgathered"]
    return all(o["allgathered"] == ref for o in outs) and len({tuple(o["allgathered"][:8]) for o in outs}) == 1


def test_elastic_shrink_after_worker_failure(tmp_path):
    p, outs = run(tmp_path, "shrink", ["-np", "3", "--min-np", "2"])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert "continuing with 2 workers" in p.stderr
    assert sorted(o["wid"] for o in outs) == [0, 1]
    for o in outs:
        assert o["step"] == 24 and o["size"] == 2 and o["resets"] == 1
        # rolled back to the step-8 commit: steps 1-8 ran with 3 workers, 9-24 with 2
        assert o["sizes"] == [3] * 8 + [2] * 16, o["sizes"]
    assert _consistent(outs)


def test_elastic_respawn_replaces_worker(tmp_path):
    p, outs = run(tmp_path, "respawn", ["-np", "3", "--min-np", "2", "--respawn"])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert "respawned as worker 3" in p.stderr
    assert sorted(o["wid"] for o in outs) == [0, 1, 3]
    for o in outs:
        assert o["step"] == 24 and o["size"] == 3
        assert o["sizes"] == [3] * 24  # the replacement received the committed state and history
    assert _consistent(outs)


def test_elastic_grow_on_request(tmp_path):
    p, outs = run(tmp_path, "grow", ["-np", "2", "--min-np", "2", "--max-np", "3"])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert sorted(o["wid"] for o in outs) == [0, 1, 2]
    for o in outs:
        assert o["step"] == 24 and o["size"] == 3
        assert o["sizes"][:6] == [2] * 6 and o["sizes"][-1] == 3
    assert _consistent(outs)


def test_elastic_below_min_np_aborts(tmp_path):
    p, _ = run(tmp_path, "shrink", ["-np", "3", "--min-np", "3"])
    assert p.returncode == 3
    assert "fewer than --min-np 3" in p.stderr
