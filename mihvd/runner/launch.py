"""``mihvdrun`` — an mpirun/horovodrun-compatible launcher.

The reference's MPIJob launcher runs (horovod/tensorflow-mnist.yaml:17-38)::

    mpirun -np 2 --allow-run-as-root -bind-to none -map-by slot -x LD_LIBRARY_PATH -x PATH \
           -mca pml ob1 -mca btl ^openib python /examples/tensorflow_mnist.py

``mihvdrun`` accepts exactly that argv (plus horovodrun's ``-np N -H host:slots``). MPI transport
flags (``-mca``, ``-bind-to``) are accepted and ignored — the data plane is RCCL over xGMI, the
bootstrap is the launcher's own C++ key-value store (``MIHVD_STORE_ADDR``, mihvd/runner/store.py;
``MIHVD_STORE=torch`` falls back to torch's TCPStore at ``MASTER_ADDR:MASTER_PORT``). Ranks are laid out by
``-map-by slot`` (fill each host) or ``-map-by node`` (round robin); local ranks on a host get
consecutive GPUs. Remote hosts are reached over ssh, as mpirun does inside an MPIJob (hostfile from
``--hostfile`` or ``$OMPI_MCA_orte_default_hostfile``, which the MPI Operator mounts).

Each rank receives ``RANK WORLD_SIZE LOCAL_RANK LOCAL_WORLD_SIZE GROUP_RANK MASTER_ADDR
MASTER_PORT`` and the Open MPI equivalents ``OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE}``.
If any rank exits non-zero the others are terminated and that exit code is returned (mpirun
semantics: one dead rank aborts the job) — unless the job is elastic (``--min-np M [--max-np N]
[--respawn]``, see mihvd/elastic.py): then the launcher publishes a new membership generation
without the dead worker (or with a replacement) and only aborts below M workers; SIGUSR1 asks it to
add a worker (up to N).
"""
from __future__ import annotations

import argparse
import os
import shlex
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field

_IGNORED_WITH_ARG = {"-bind-to", "--bind-to", "-map-by", "--map-by", "-rank-by", "--rank-by", "--prefix", "-prefix",
                     "-wdir", "--wdir", "-wd", "--network-interface", "--network-interfaces", "--gloo-timeout-seconds",
                     "--config-file"}
_IGNORED_FLAGS = {"--allow-run-as-root", "-allow-run-as-root", "--oversubscribe", "-oversubscribe",
                  "--report-bindings", "-report-bindings", "--display-map", "-display-map", "-q", "--quiet",
                  "--gloo", "--mpi", "--nccl", "--rccl", "--use-hwthread-cpus", "-use-hwthread-cpus",
                  "--bind-to-core", "-bind-to-core", "--enable-recovery", "-v", "--disable-cache",
                  "--mpi-threads-disable"}


@dataclass
class LaunchSpec:
    np: int = 1
    hosts: list[tuple[str, int]] = field(default_factory=list)
    map_by: str = "slot"
    env_forward: dict[str, str | None] = field(default_factory=dict)
    mca: list[tuple[str, str]] = field(default_factory=list)
    ignored: list[str] = field(default_factory=list)
    tag_output: bool = False
    master_addr: str | None = None
    master_port: int | None = None
    ssh_port: int | None = None
    extra_env: dict[str, str] = field(default_factory=dict)
    start_timeout: float = 120.0
    min_np: int | None = None          # elastic (mihvd.elastic): keep going while >= min_np workers live
    max_np: int | None = None
    respawn: bool = False              # elastic: replace a dead worker (same slot) with a new one
    verbose: bool = False
    output_dir: str | None = None      # mpirun --output-filename: rank r's output also goes to <dir>/1/rank.r/
    command: list[str] = field(default_factory=list)


def parse_hosts(spec: str) -> list[tuple[str, int]]:
    out = []
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        if ":" in item:
            h, s = item.rsplit(":", 1)
            out.append((h, int(s)))
        else:
            out.append((item, 1))
    return out


def parse_hostfile(path: str) -> list[tuple[str, int]]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            parts = line.split()
            host, slots = parts[0], 1
            if ":" in host:
                host, s = host.rsplit(":", 1)
                slots = int(s)
            for p in parts[1:]:
                if p.startswith("slots="):
                    slots = int(p.split("=", 1)[1])
            out.append((host, slots))
    return out


def parse_args(argv: list[str]) -> LaunchSpec:
    """Hand-rolled parser: mpirun mixes single-dash long options with GNU style."""
    spec = LaunchSpec()
    i = 0
    n = len(argv)
    hostfile = None
    np_given = False

    def need(k):
        if i + 1 >= n:
            raise SystemExit(f"mihvdrun: option {k} needs an argument")
        return argv[i + 1]

    while i < n:
        a = argv[i]
        if a == "--":
            spec.command = argv[i + 1:]
            break
        if a in ("-np", "--np", "-n", "-c"):
            spec.np = int(need(a)); np_given = True; i += 2; continue
        if a.startswith("-np="):
            spec.np = int(a.split("=", 1)[1]); np_given = True; i += 1; continue
        if a in ("-H", "--host", "-host", "--hosts"):
            spec.hosts = parse_hosts(need(a)); i += 2; continue
        if a in ("--hostfile", "-hostfile", "--machinefile", "-machinefile", "-hf"):
            hostfile = need(a); i += 2; continue
        if a in ("-map-by", "--map-by"):
            spec.map_by = need(a).split(":", 1)[0].lower(); spec.ignored.append(f"{a} {argv[i + 1]}"); i += 2; continue
        if a in ("-x",):
            kv = need(a)
            if "=" in kv:
                k, v = kv.split("=", 1)
                spec.env_forward[k] = v
            else:
                spec.env_forward[kv] = None
            i += 2; continue
        if a in ("-mca", "--mca", "-gmca", "--gmca"):
            if i + 2 >= n:
                raise SystemExit(f"mihvdrun: {a} needs two arguments")
            spec.mca.append((argv[i + 1], argv[i + 2])); i += 3; continue
        if a in ("--tag-output", "-tag-output"):
            spec.tag_output = True; i += 1; continue
        if a in ("--master-addr", "--master_addr"):
            spec.master_addr = need(a); i += 2; continue
        if a in ("--master-port", "--master_port"):
            spec.master_port = int(need(a)); i += 2; continue
        if a in ("-p", "--ssh-port"):
            spec.ssh_port = int(need(a)); i += 2; continue
        if a in ("--start-timeout",):
            spec.start_timeout = float(need(a)); i += 2; continue
        if a in ("--verbose",):
            spec.verbose = True; i += 1; continue
        if a in ("--min-np", "--min_np"):
            spec.min_np = int(need(a)); i += 2; continue
        if a in ("--max-np", "--max_np"):
            spec.max_np = int(need(a)); i += 2; continue
        if a in ("--respawn", "--elastic-respawn"):
            spec.respawn = True; i += 1; continue
        if a in ("--timeline-filename",):
            spec.extra_env["MIHVD_TIMELINE"] = need(a); i += 2; continue
        if a in ("--fusion-threshold-mb",):
            spec.extra_env["MIHVD_FUSION_THRESHOLD"] = str(int(float(need(a)) * 1024 * 1024)); i += 2; continue
        if a in ("--cycle-time-ms",):
            spec.extra_env["MIHVD_CYCLE_TIME"] = need(a); i += 2; continue
        if a in ("--stall-check-warning-time-seconds",):
            spec.extra_env["MIHVD_STALL_CHECK_TIME_SECONDS"] = need(a); i += 2; continue
        if a in ("--stall-check-shutdown-time-seconds",):
            spec.extra_env["MIHVD_STALL_SHUTDOWN_TIME_SECONDS"] = need(a); i += 2; continue
        if a in ("--no-stall-check",):
            spec.extra_env["MIHVD_STALL_CHECK_DISABLE"] = "1"; i += 1; continue
        if a in ("--hierarchical-allreduce",):
            spec.extra_env["MIHVD_HIERARCHICAL_ALLREDUCE"] = "1"; i += 1; continue
        if a in ("--autotune",):
            spec.extra_env["MIHVD_AUTOTUNE"] = "1"; i += 1; continue
        if a in ("--autotune-log-file",):
            spec.extra_env["MIHVD_AUTOTUNE_LOG"] = need(a); i += 2; continue
        if a in ("--log-level",):
            spec.extra_env["MIHVD_LOG_LEVEL"] = need(a).upper(); i += 2; continue
        if a in ("--output-filename", "-output-filename"):
            spec.output_dir = need(a); i += 2; continue
        if a in _IGNORED_WITH_ARG:
            spec.ignored.append(f"{a} {need(a)}"); i += 2; continue
        if a in _IGNORED_FLAGS:
            spec.ignored.append(a); i += 1; continue
        if a.startswith("-"):
            raise SystemExit(f"mihvdrun: unknown option {a}")
        spec.command = argv[i:]
        break
    if not spec.command:
        raise SystemExit("mihvdrun: no command given")
    if hostfile is None and not spec.hosts and os.environ.get("OMPI_MCA_orte_default_hostfile"):
        hostfile = os.environ["OMPI_MCA_orte_default_hostfile"]
    if hostfile:
        spec.hosts = parse_hostfile(hostfile)
    if not spec.hosts:
        spec.hosts = [("localhost", spec.np)]
    if not np_given:
        spec.np = sum(s for _, s in spec.hosts)
    return spec


def assign_ranks(hosts: list[tuple[str, int]], np_: int, map_by: str = "slot"):
    """Returns [(rank, host, local_rank, local_size, node_index)]."""
    total = sum(s for _, s in hosts)
    if np_ > total:
        raise SystemExit(f"mihvdrun: -np {np_} exceeds the {total} slots available on {hosts}")
    per_host: list[list[int]] = [[] for _ in hosts]
    if map_by == "node":
        r = 0
        while r < np_:
            for h, (_, slots) in enumerate(hosts):
                if r < np_ and len(per_host[h]) < slots:
                    per_host[h].append(r)
                    r += 1
    else:
        r = 0
        for h, (_, slots) in enumerate(hosts):
            take = min(slots, np_ - r)
            per_host[h].extend(range(r, r + take))
            r += take
    out = []
    node = 0
    for h, ranks in enumerate(per_host):
        if not ranks:
            continue
        for lr, rank in enumerate(ranks):
            out.append((rank, hosts[h][0], lr, len(ranks), node))
        node += 1
    return sorted(out)


def _is_local(host: str) -> bool:
    if host in ("localhost", "127.0.0.1", "::1"):
        return True
    try:
        return host in (socket.gethostname(), socket.getfqdn())
    except Exception:
        return False


def _free_port(addr="127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr if addr != "localhost" else "127.0.0.1", 0))
        return s.getsockname()[1]


# Variables forwarded to every rank by default, like horovodrun (which forwards the launcher's
# environment): the framework's and Horovod's knobs, the collective library's, the ROCm runtime's
# and the Python path. mpirun forwards only its -x list; in an MPIJob the ranks on the worker pods
# are started over ssh, whose sessions do not inherit the container's Docker ENV, so the settings
# an operator puts on the launcher must travel with the command. MIHVD_FORWARD_PREFIXES overrides
# the list ("" forwards nothing beyond -x); *_VISIBLE_DEVICES is never forwarded (the launcher
# pod's GPU view is not the worker's).
DEFAULT_FORWARD_PREFIXES = ("MIHVD_", "HOROVOD_", "NCCL_", "RCCL_", "HSA_", "HIP_", "ROCR_", "TORCH_NCCL_",
                            "PYTORCH_", "OMP_NUM_THREADS", "PYTHONPATH")
_NEVER_FORWARD = ("MIHVD_LAUNCHED", "MIHVD_STORE_ADDR", "MIHVD_WORKER_ID", "MIHVD_ELASTIC", "MIHVD_DEVICE_INDEX")


def forward_prefixes(base=None) -> tuple[str, ...]:
    base = os.environ if base is None else base
    v = base.get("MIHVD_FORWARD_PREFIXES")
    if v is None:
        return DEFAULT_FORWARD_PREFIXES
    return tuple(p.strip() for p in v.split(",") if p.strip())


def build_rank_env(spec: LaunchSpec, rank, local_rank, local_size, node, master_addr, master_port, base_env=None):
    base = dict(os.environ if base_env is None else base_env)
    env = {}
    pre = forward_prefixes(base)
    for k, v in base.items():
        if (pre and k.startswith(pre) and not k.endswith("_VISIBLE_DEVICES") and k not in _NEVER_FORWARD
                and k != "MIHVD_FORWARD_PREFIXES"):
            env[k] = v
    for k, v in spec.env_forward.items():
        if v is not None:
            env[k] = v
        elif k in base:
            env[k] = base[k]
    env.update(spec.extra_env)
    env.update({
        "RANK": str(rank), "WORLD_SIZE": str(spec.np), "LOCAL_RANK": str(local_rank),
        "LOCAL_WORLD_SIZE": str(local_size), "GROUP_RANK": str(node), "MASTER_ADDR": master_addr,
        "MASTER_PORT": str(master_port), "OMPI_COMM_WORLD_RANK": str(rank), "OMPI_COMM_WORLD_SIZE": str(spec.np),
        "OMPI_COMM_WORLD_LOCAL_RANK": str(local_rank), "OMPI_COMM_WORLD_LOCAL_SIZE": str(local_size),
        "MIHVD_LAUNCHED": "1",
    })
    return env


def remote_command(spec: LaunchSpec, renv: dict[str, str], cwd: str | None = None) -> str:
    """The shell command a remote rank runs (after ssh): cd to the launcher's working directory,
    then the program under exactly ``renv`` on top of the ssh session's own environment."""
    exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in renv.items())
    return (f"cd {shlex.quote(cwd or os.getcwd())} && env {exports} " +
            " ".join(shlex.quote(c) for c in spec.command))


def ssh_command(spec: LaunchSpec, host: str, renv: dict[str, str]) -> list[str]:
    return (["ssh", "-o", "StrictHostKeyChecking=no"] + (["-p", str(spec.ssh_port)] if spec.ssh_port else []) +
            [host, remote_command(spec, renv)])


class _Proc:
    def __init__(self, rank, popen):
        self.rank = rank
        self.popen = popen


def _pump(stream, out, prefix, copy_path=None):
    copy = open(copy_path, "ab") if copy_path else None
    try:
        for line in iter(stream.readline, b""):
            if prefix:
                out.buffer.write(prefix.encode() + line)
            else:
                out.buffer.write(line)
            out.flush()
            if copy is not None:
                copy.write(line)
                copy.flush()
    finally:
        stream.close()
        if copy is not None:
            copy.close()


def launch(spec: LaunchSpec) -> int:
    layout = assign_ranks(spec.hosts, spec.np, spec.map_by)
    first_host = layout[0][1]
    all_local = all(_is_local(h) for _, h, *_ in layout)
    master_addr = spec.master_addr or ("127.0.0.1" if all_local else first_host)
    master_port = spec.master_port or (_free_port() if all_local else 29500)
    if spec.verbose:
        for m in spec.ignored:
            print(f"mihvdrun: ignoring MPI option {m}", file=sys.stderr)
        for k, v in spec.mca:
            print(f"mihvdrun: ignoring MCA parameter {k}={v} (data plane is RCCL)", file=sys.stderr)
    # The rendezvous server (C++ StoreServer, csrc/runtime/store.cc) lives in the launcher, like
    # horovodrun's: ranks build their process group and the negotiation engine over it.
    elastic = spec.min_np is not None or spec.max_np is not None
    server = client = None
    if os.environ.get("MIHVD_STORE", "native") != "torch" or elastic:
        from .store import start_server

        server = start_server("127.0.0.1" if all_local else "0.0.0.0", 0)
    min_np = spec.min_np if spec.min_np is not None else spec.np
    max_np = spec.max_np if spec.max_np is not None else spec.np
    if elastic:
        from .._native import runtime
        from ..elastic import GEN_KEY, format_members, members_key

        if not 1 <= min_np <= spec.np <= max_np:
            raise SystemExit(f"mihvdrun: need 1 <= --min-np ({min_np}) <= -np ({spec.np}) <= --max-np ({max_np})")
        client = runtime().StoreClient("127.0.0.1" if all_local else master_addr, server.port, 30.0)
    procs: list[_Proc] = []
    threads = []
    slots = {}     # worker id -> (host, local_rank, local_size, node)
    members = []   # current generation: [(worker id, host)] in rank order
    gen = [-1]

    def publish(new_members):
        gen[0] += 1
        client.set(members_key(gen[0]), format_members(new_members))
        client.set(GEN_KEY, str(gen[0]))
        if spec.verbose or gen[0] > 0:
            print(f"mihvdrun: elastic generation {gen[0]}: {len(new_members)} workers "
                  f"{[w for w, _ in new_members]}", file=sys.stderr, flush=True)

    def spawn(wid, rank, host, lr, ls, node):
        renv = build_rank_env(spec, rank, lr, ls, node, master_addr, master_port)
        if server is not None:
            renv["MIHVD_STORE_ADDR"] = f"{master_addr}:{server.port}"
        if elastic:
            renv.update({"MIHVD_ELASTIC": "1", "MIHVD_WORKER_ID": str(wid), "MIHVD_DEVICE_INDEX": str(lr),
                         "WORLD_SIZE": str(max(len(members), rank + 1)), "OMPI_COMM_WORLD_SIZE": str(max(len(members), rank + 1))})
        if _is_local(host):
            env = dict(os.environ)
            env.update(renv)
            cmd = spec.command
        else:
            cmd = ssh_command(spec, host, renv)
            env = dict(os.environ)
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True)
        procs.append(_Proc(wid, p))
        slots[wid] = (host, lr, ls, node)
        pre_o = f"[1,{wid}]<stdout>:" if spec.tag_output else ""
        pre_e = f"[1,{wid}]<stderr>:" if spec.tag_output else ""
        rank_dir = None
        if spec.output_dir:  # Open MPI's layout: <dir>/1/rank.<r>/{stdout,stderr}
            rank_dir = os.path.join(spec.output_dir, "1", f"rank.{wid}")
            os.makedirs(rank_dir, exist_ok=True)
        for st, o, pre, name in ((p.stdout, sys.stdout, pre_o, "stdout"), (p.stderr, sys.stderr, pre_e, "stderr")):
            t = threading.Thread(target=_pump, args=(st, o, pre, os.path.join(rank_dir, name) if rank_dir else None),
                                 daemon=True)
            t.start()
            threads.append(t)

    if elastic:
        publish([(rank, host) for rank, host, *_ in layout])
        members = [(rank, host) for rank, host, *_ in layout]
    for rank, host, lr, ls, node in layout:
        spawn(rank, rank, host, lr, ls, node)

    def terminate_all(sig=signal.SIGTERM):
        for pr in procs:
            if pr.popen.poll() is None:
                try:
                    os.killpg(pr.popen.pid, sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, frame):
        terminate_all(signal.SIGTERM)

    def abort(code, why):
        print(f"mihvdrun: {why}; terminating the job", file=sys.stderr, flush=True)
        terminate_all(signal.SIGTERM)
        deadline = time.time() + 10
        while time.time() < deadline and any(p.popen.poll() is None for p in procs):
            time.sleep(0.05)
        terminate_all(signal.SIGKILL)
        return code

    grow = [0]

    def on_grow(signum, frame):  # elastic scale-up request (e.g. from a host-discovery hook)
        grow[0] += 1

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGINT, signal.SIGTERM)}
    if elastic:
        old[signal.SIGUSR1] = signal.signal(signal.SIGUSR1, on_grow)
    exit_code = 0
    succeeded = 0
    next_wid = spec.np
    try:
        remaining = set(range(len(procs)))
        while remaining:
            while elastic and grow[0] > 0 and not succeeded and exit_code == 0:
                grow[0] -= 1
                if len(members) >= max_np:
                    print(f"mihvdrun: scale-up ignored: already --max-np {max_np} workers", file=sys.stderr, flush=True)
                    continue
                host, lr, ls, node = slots[members[0][0]]
                lr = len(members) % max(1, ls)
                new = next_wid
                next_wid += 1
                members.append((new, host))
                publish(members)
                spawn(new, len(members) - 1, host, lr, ls, node)
                remaining.add(len(procs) - 1)
            for i in list(remaining):
                rc = procs[i].popen.poll()
                if rc is None:
                    continue
                remaining.discard(i)
                wid = procs[i].rank
                if rc == 0:
                    succeeded += 1
                    continue
                code = rc if rc > 0 else 128 - rc
                if not elastic or succeeded:
                    if exit_code == 0:
                        exit_code = abort(code, f"rank {wid} exited with code {rc}")
                    continue
                # elastic: drop the dead worker (optionally replace it) and publish a new generation
                members = [(w, h) for w, h in members if w != wid]
                if spec.respawn and len(members) < max_np:
                    host, lr, ls, node = slots[wid]
                    new = next_wid
                    next_wid += 1
                    members.append((new, host))
                    publish(members)
                    spawn(new, len(members) - 1, host, lr, ls, node)
                    remaining.add(len(procs) - 1)
                    print(f"mihvdrun: worker {wid} exited with code {rc}; respawned as worker {new}",
                          file=sys.stderr, flush=True)
                elif len(members) >= min_np:
                    print(f"mihvdrun: worker {wid} exited with code {rc}; continuing with {len(members)} workers "
                          f"(--min-np {min_np})", file=sys.stderr, flush=True)
                    publish(members)
                elif exit_code == 0:
                    exit_code = abort(code, f"worker {wid} exited with code {rc} and fewer than --min-np {min_np} "
                                            "workers remain")
            time.sleep(0.02)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
        for t in threads:
            t.join(timeout=5)
        if client is not None:
            client.close()
        if server is not None:
            server.stop()
    return exit_code


def check_build() -> str:
    """``horovodrun --check-build``: what this installation can run (frameworks, controllers,
    tensor operations), probed without initialising a GPU."""
    import importlib.util

    def box(ok):
        return "[X]" if ok else "[ ]"

    try:
        import torch
        torch_ok = True
        rocm = getattr(torch.version, "hip", None) is not None
        dist_ok = torch.distributed.is_available()
        nccl = dist_ok and torch.distributed.is_nccl_available()
        gloo = dist_ok and torch.distributed.is_gloo_available()
        mpi = dist_ok and torch.distributed.is_mpi_available()
    except Exception:  # pragma: no cover
        torch_ok = rocm = nccl = gloo = mpi = False
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    native = os.path.isdir(os.path.join(here, "_native"))
    kernels = native and os.path.exists(os.path.join(here, "_native", "libmihvd_kernels.so"))
    runtime = native and any(f.startswith("_mihvd_runtime") for f in os.listdir(os.path.join(here, "_native")))
    from .. import __version__

    lines = [f"mihvd v{__version__}:", "", "Available Frameworks:",
             f"    {box(torch_ok)} PyTorch{' (ROCm)' if rocm else ''}  (mihvd.torch)",
             f"    {box(torch_ok)} TensorFlow-shaped API on PyTorch  (mihvd.tensorflow: hooks, MonitoredTrainingSession)",
             f"    {box(torch_ok)} Keras-shaped API on PyTorch  (mihvd.keras: callbacks, fit)",
             f"    {box(importlib.util.find_spec('mxnet') is not None)} MXNet",
             "", "Available Controllers:",
             f"    {box(runtime)} native C++ store + negotiation engine",
             f"    {box(gloo)} Gloo", f"    {box(mpi)} MPI",
             "", "Available Tensor Operations:",
             f"    {box(nccl and rocm)} RCCL  (torch.distributed 'nccl' backend on ROCm)",
             f"    {box(kernels)} direct xGMI (hipIpc peer memory, csrc/kernels/xgmi.hip)",
             f"    {box(kernels)} CDNA4 HIP kernels (gfx950: fused MNIST step, multi-tensor optimizers, Adasum)",
             f"    {box(gloo)} Gloo", f"    {box(mpi)} MPI", f"    {box(False)} DDL", f"    {box(False)} CCL"]
    return "\n".join(lines)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if argv and argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    if argv and argv[0] in ("-cb", "--check-build"):
        print(check_build())
        return 0
    spec = parse_args(argv)
    return launch(spec)


if __name__ == "__main__":
    sys.exit(main())
