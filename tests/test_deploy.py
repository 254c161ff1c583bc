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


def test_mi355x_mpijob():
    (job,) = _load("mpijob-mi355x.yaml")
    worker = _check_mpijob(job, 8, 8)
    c = worker["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    vols = {v["name"]: v for v in worker["template"]["spec"]["volumes"]}
    assert vols["checkpoints"]["persistentVolumeClaim"]["claimName"] == "mihvd-checkpoints"


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


def test_elastic_mpijob():
    (job,) = _load("mpijob-mi355x-elastic.yaml")
    spec = job["spec"]
    assert job["apiVersion"] == "kubeflow.org/v2beta1" and spec["slotsPerWorker"] == 8
    c = spec["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    ls = L.parse_args([str(a) for a in c["args"]])
    assert (ls.np, ls.min_np, ls.max_np, ls.respawn) == (16, 8, 16, True)
    assert ls.command[:2] == ["python", "/examples/tensorflow_mnist_elastic.py"]
    assert spec["mpiReplicaSpecs"]["Worker"]["replicas"] * 8 >= ls.max_np
