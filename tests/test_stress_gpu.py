"""BASELINE.json stretch configs run end to end on one MI355X through mihvd's DistributedOptimizer
(ResNet-50 bf16; BERT-base MLM seq 512 with fp16 allreduce compression)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("model,extra", [("resnet50", ["--batch-size", "32"]),
                                         ("bert-base", ["--batch-size", "4", "--graph", "--steps", "6"])])
def test_stress_model_runs(model, extra):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "stress_models.py"), "--model", model,
                        "--steps", "3", "--warmup", "3", *extra], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["value"] > 0 and rec["n_gpus"] == 1
    assert rec["config"]["final_loss"] == rec["config"]["final_loss"]  # not NaN
