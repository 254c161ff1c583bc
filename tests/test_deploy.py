"""Deployment artifacts: MPIJob manifests (kubeflow.org/v2beta1 shape), launcher argv in them,
deploy script syntax and dry run (no cluster is available in CI)."""
import os
import subprocess

import yaml

from mihvd.runner import launch as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def _load(name):
    with open(os.path.join(DEPLOY, name)) as f:
        return list(yaml.safe_load_all(f))


def _check_mpijob(job, np_, slots):
    assert job["apiVersion"] == "kubeflow.org/v2beta1" and job["kind"] == "MPIJob"
    spec = job["spec"]
    assert spec["slotsPerWorker"] == slots
    assert spec["runPolicy"]["cleanPodPolicy"] == "Running"
    launcher = spec["mpiReplicaSpecs"]["Launcher"]
    worker = spec["mpiReplicaSpecs"]["Worker"]
    assert launcher["replicas"] == 1
    c = launcher["template"]["spec"]["containers"][0]
    assert c["command"] == ["mihvdrun"]
    ls = L.parse_args([str(a) for a in c["args"]])
    assert ls.np == np_ and ls.command[:2] == ["python", "/examples/tensorflow_mnist.py"]
    assert worker["replicas"] * slots >= np_
    return worker


def _rank_env_of(job):
    """The environment a rank on a worker pod receives: mihvdrun's forwarded set, built from the
    launcher container's env (the only env that reaches an ssh-started rank)."""
    launcher = job["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    ls = L.parse_args([str(a) for a in launcher["args"]])
    lenv = {"PATH": "/usr/bin:/bin", "LD_LIBRARY_PATH": "/opt/rocm/lib"}
    lenv.update({e["name"]: str(e["value"]) for e in launcher.get("env", [])})
    return ls, L.build_rank_env(ls, 9, 1, 8, 1, "10.0.0.1", 29500, base_env=lenv)


def test_mi355x_mpijob():
    (job,) = _load("mpijob-mi355x.yaml")
    worker = _check_mpijob(job, 8, 8)
    c = worker["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    # settings on the worker container would only reach its sshd, never an ssh-started rank
    assert not c.get("env"), "put rank settings on the launcher (mihvdrun forwards them)"
    ls, renv = _rank_env_of(job)
    assert renv["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert renv["MIHVD_STALL_CHECK_TIME_SECONDS"] == "60" and renv["MIHVD_STALL_SHUTDOWN_TIME_SECONDS"] == "600"
    assert "MIHVD_STALL_CHECK_TIME_SECONDS" in ls.env_forward
    assert renv["RANK"] == "9" and renv["LOCAL_RANK"] == "1"
    vols = {v["name"]: v for v in worker["template"]["spec"]["volumes"]}
    assert vols["checkpoints"]["persistentVolumeClaim"]["claimName"] == "mihvd-checkpoints"


def test_mpijob_rank_env_starts_no_engine_thread():
    """At N > 1 on RCCL the job's ranks start no background engine (the fused trainer issues its
    own collectives; a second communicator cycling beside it could deadlock)."""
    from mihvd.basics import engine_wanted
    from mihvd.config import Config

    for name in ("mpijob-mi355x.yaml", "mpijob-mi355x-elastic.yaml"):
        (job,) = _load(name)
        _, renv = _rank_env_of(job)
        assert not engine_wanted(Config.from_env(renv), 8, "nccl"), name
    assert not engine_wanted(Config.from_env({}), 8, "nccl")
    assert engine_wanted(Config.from_env({"MIHVD_ENGINE": "native"}), 8, "nccl")
    assert engine_wanted(Config.from_env({"MIHVD_NEGOTIATE": "1"}), 2, "gloo")


def test_launcher_forwards_framework_env_by_default():
    """horovodrun-style forwarding: MIHVD_* / HOROVOD_* / NCCL_* / HSA_* and PYTHONPATH reach every
    rank without -x; *_VISIBLE_DEVICES and launcher-private variables do not; MIHVD_FORWARD_PREFIXES
    narrows it."""
    ls = L.parse_args(["-np", "2", "-x", "FOO", "python", "x.py"])
    base = {"MIHVD_X": "1", "HOROVOD_FUSION_THRESHOLD": "2", "NCCL_DEBUG": "INFO", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            "PYTHONPATH": "/opt/mihvd", "HIP_VISIBLE_DEVICES": "3", "MIHVD_STORE_ADDR": "a:1", "FOO": "f",
            "UNRELATED": "u"}
    env = L.build_rank_env(ls, 1, 1, 2, 0, "127.0.0.1", 1234, base_env=base)
    for k in ("MIHVD_X", "HOROVOD_FUSION_THRESHOLD", "NCCL_DEBUG", "HSA_ENABLE_IPC_MODE_LEGACY", "PYTHONPATH", "FOO"):
        assert env[k] == base[k], k
    for k in ("HIP_VISIBLE_DEVICES", "MIHVD_STORE_ADDR", "UNRELATED"):
        assert k not in env, k
    env = L.build_rank_env(ls, 1, 1, 2, 0, "127.0.0.1", 1234, base_env=dict(base, MIHVD_FORWARD_PREFIXES=""))
    assert "MIHVD_X" not in env and env["FOO"] == "f"


def test_remote_rank_command_imports_mihvd_without_inherited_env(tmp_path):
    """The command an ssh-started rank runs (launch.remote_command) under an EMPTY environment
    (`env -i`, as an ssh session on a worker pod: no Docker ENV): the launcher's forwarded set alone
    makes mihvd importable and carries the rank's settings."""
    import sys

    ls = L.parse_args(["-np", "2", "-x", "PATH", sys.executable, "-c",
                       "import os, mihvd, mihvd.runner; print('OK', os.environ['RANK'], "
                       "os.environ['MIHVD_STALL_CHECK_TIME_SECONDS'])"])
    base = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "PYTHONPATH": ROOT, "MIHVD_STALL_CHECK_TIME_SECONDS": "60"}
    renv = L.build_rank_env(ls, 1, 1, 2, 1, "127.0.0.1", 1234, base_env=base)
    cmd = L.remote_command(ls, renv, cwd=str(tmp_path))
    out = subprocess.run(["env", "-i", "sh", "-c", cmd], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["OK", "1", "60"], out.stdout


def test_cpu_mpijob_matches_reference_topology():
    (job,) = _load("mpijob-cpu.yaml")
    worker = _check_mpijob(job, 2, 1)
    assert worker["replicas"] == 2
    args = job["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]["args"]
    ls = L.parse_args([str(a) for a in args])
    assert ls.env_forward["MIHVD_BACKEND"] == "gloo"
    assert ("btl", "^openib") in ls.mca


def test_pvc():
    (pvc,) = _load("checkpoint-pvc.yaml")
    assert pvc["kind"] == "PersistentVolumeClaim" and pvc["metadata"]["name"] == "mihvd-checkpoints"


def test_deploy_script_dry_run():
    script = os.path.join(DEPLOY, "deploy_stack.sh")
    assert subprocess.run(["bash", "-n", script]).returncode == 0
    out = subprocess.run(["bash", script], env={**os.environ, "DRY_RUN": "1", "IMAGE": "reg/mihvd:1"},
                         capture_output=True, text=True, check=True).stdout
    assert "kubectl create namespace ml-ops" in out and "kubectl create namespace loki" in out
    assert "helm upgrade --install loki grafana/loki-stack" in out and "loki.persistence.size=5Gi" in out
    assert "mpi-operator/v0.6.0/deploy/v2beta1/mpi-operator.yaml" in out  # pinned, not master
    assert "reg/mihvd:1" in out


def test_dockerfile_builds_native_for_gfx950():
    text = open(os.path.join(DEPLOY, "Dockerfile")).read()
    assert "mihvd._build all" in text and "gfx950" in text and "openssh-server" in text
    # installed site-wide (a .pth in site-packages), not through Docker ENV, which ssh-started ranks
    # never see
    assert "mihvd.pth" in text and "site.getsitepackages()" in text
    assert "ENV PYTHONPATH" not in text


def test_elastic_mpijob():
    (job,) = _load("mpijob-mi355x-elastic.yaml")
    spec = job["spec"]
    assert job["apiVersion"] == "kubeflow.org/v2beta1" and spec["slotsPerWorker"] == 8
    c = spec["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    ls = L.parse_args([str(a) for a in c["args"]])
    assert (ls.np, ls.min_np, ls.max_np, ls.respawn) == (16, 8, 16, True)
    assert ls.command[:2] == ["python", "/examples/tensorflow_mnist_elastic.py"]
    assert spec["mpiReplicaSpecs"]["Worker"]["replicas"] * 8 >= ls.max_np


def _logql_regexes(expr):
    """The RE2 patterns inside `...` of a LogQL query (`regexp` stages and `|~` filters)."""
    import re

    return re.findall(r"`([^`]*)`", expr)


def test_loki_values_and_dashboard_parse_the_training_logs():
    """Promtail's rank-label stage and every Grafana panel query match the lines the framework
    writes (mihvd/utils/logging.py via LoggingTensorHook / StepCounterHook)."""
    import json
    import re

    from mihvd.utils.logging import fmt_kv

    (vals,) = _load("loki-stack-values.yaml")
    assert vals["loki"]["persistence"] == {"enabled": True, "size": "5Gi"}
    assert vals["grafana"]["sidecar"]["dashboards"]["label"] == "grafana_dashboard"
    stages = vals["promtail"]["config"]["snippets"]["pipelineStages"]
    match = [s["match"] for s in stages if "match" in s][0]
    rx = [s["regex"]["expression"] for s in match["stages"] if "regex" in s][0]
    lines = ["[rank 3/8] " + fmt_kv(step=120, loss=0.0421, sec=0.012),
             "[rank 0/8] " + fmt_kv(**{"global_step/sec": 14210.5, "img_per_sec": 11368400.0}),
             "[rank 1/8] " + fmt_kv(step=7, val_loss=9.5, loss=1.5)]
    m = re.match(rx, lines[0])
    assert m and m.group("rank") == "3" and m.group("world") == "8"

    dash = json.load(open(os.path.join(DEPLOY, "grafana", "mihvd-dashboard.json")))
    assert dash["uid"] == "mihvd-mnist" and len(dash["panels"]) >= 5
    want = {"loss": {0: 0.0421, 2: 1.5}, "step": {0: 120.0, 2: 7.0}, "img_per_sec": {1: 11368400.0},
            "global_step/sec": {1: 14210.5}}
    seen = set()
    for p in dash["panels"]:
        for t in p["targets"]:
            for pat in _logql_regexes(t["expr"]):
                if "(?P<v>" not in pat:
                    assert re.search(pat, "[rank 1/8] RuntimeError: stall detected")
                    continue
                key = re.search(r"\)(.+)=\(\?P<v>", pat).group(1)
                seen.add(key)
                for i, line in enumerate(lines):
                    m = re.search(pat, line)
                    if i in want[key]:
                        assert m and float(m.group("v")) == want[key][i], (key, line)
                    else:
                        assert m is None, (key, line)   # `loss` never picks up `val_loss`
    assert seen == set(want)


def test_deploy_script_provisions_dashboard():
    out = subprocess.run(["bash", os.path.join(DEPLOY, "deploy_stack.sh")], env={**os.environ, "DRY_RUN": "1"},
                         capture_output=True, text=True, check=True).stdout
    assert "-f " in out and "loki-stack-values.yaml" in out
    assert "create configmap mihvd-dashboard -n loki" in out and "grafana_dashboard=1" in out
