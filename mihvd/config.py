"""Engine configuration: one frozen dataclass resolved at ``init()``.

Every knob is read from ``MIHVD_<NAME>`` and, for Horovod users, from the equivalent
``HOROVOD_<NAME>`` alias (the reference forwards no such variables — tensorflow-mnist.yaml:27-30 —
so defaults apply there too).
"""
from __future__ import annotations

import dataclasses
import os

_ALIASES = {
    "FUSION_THRESHOLD": "HOROVOD_FUSION_THRESHOLD",
    "CYCLE_TIME": "HOROVOD_CYCLE_TIME",
    "TIMELINE": "HOROVOD_TIMELINE",
    "STALL_CHECK_TIME_SECONDS": "HOROVOD_STALL_CHECK_TIME_SECONDS",
    "STALL_SHUTDOWN_TIME_SECONDS": "HOROVOD_STALL_SHUTDOWN_TIME_SECONDS",
    "STALL_CHECK_DISABLE": "HOROVOD_STALL_CHECK_DISABLE",
    "HIERARCHICAL_ALLREDUCE": "HOROVOD_HIERARCHICAL_ALLREDUCE",
    "AUTOTUNE": "HOROVOD_AUTOTUNE",
    "AUTOTUNE_LOG": "HOROVOD_AUTOTUNE_LOG",
    "LOG_LEVEL": "HOROVOD_LOG_LEVEL",
    "NEGOTIATE": "HOROVOD_NEGOTIATE",
}


def _get(name, default, cast, env):
    for key in ("MIHVD_" + name, _ALIASES.get(name)):
        if key and env.get(key) not in (None, ""):
            v = env[key]
            if cast is bool:
                return v.strip().lower() in ("1", "true", "yes", "on")
            return cast(v)
    return default


@dataclasses.dataclass(frozen=True)
class Config:
    backend: str = "auto"                 # auto | nccl (=RCCL on ROCm) | gloo
    fusion_threshold: int = 64 * 1024 * 1024  # bytes per fusion bucket (Horovod default 64 MiB)
    bucket_align: int = 256               # bytes; every gradient view starts 256-B aligned
    cycle_time_ms: float = 1.0            # HOROVOD_CYCLE_TIME compatibility (the negotiator pushes, it does not poll)
    timeline: str = ""                    # Chrome-trace path; "{rank}" is substituted
    stall_check_s: float = 60.0
    stall_shutdown_s: float = 0.0
    stall_check_disable: bool = False
    hierarchical_allreduce: bool = False
    adasum_flat: bool = False             # flat all-rank Adasum instead of hierarchical
    consistency_check: bool = True        # compare gradient signatures across ranks once
    fault: str = ""                       # fault-injection spec (tests)
    log_level: str = "INFO"
    timeout_s: float = 600.0              # process-group timeout
    autotune: bool = False                # grid-search the fusion threshold during the first steps
    autotune_candidates: str = "1,4,16,64"  # MiB
    autotune_warmup_steps: int = 3
    autotune_trial_steps: int = 8
    autotune_log: str = ""                # horovodrun --autotune-log-file: CSV of the candidates
    roctx: bool = False                   # roctx ranges around collectives / steps (rocprofv3 --marker-trace)
    negotiate: bool = False               # route async collectives through the native negotiation engine
    engine: str = "auto"                  # auto = torch (no engine thread) | native (C++ engine thread over RCCL) | python (negotiator + executor thread, MIHVD_NEGOTIATE) | torch (no engine)
    store: str = "native"                 # rendezvous: native (mihvdrun's C++ store, if present) | torch
    debug_sync: bool = False              # serialized bisection mode: sync after every kernel / collective
    elastic_grace_s: float = 30.0         # elastic: how long a failed collective waits for a new membership
    elastic_timeout_s: float = 600.0      # elastic: how long a worker waits to be included in a generation

    @staticmethod
    def from_env(env=None) -> "Config":
        env = os.environ if env is None else env
        return Config(
            backend=_get("BACKEND", "auto", str, env),
            fusion_threshold=_get("FUSION_THRESHOLD", 64 * 1024 * 1024, int, env),
            bucket_align=_get("BUCKET_ALIGN", 256, int, env),
            cycle_time_ms=_get("CYCLE_TIME", 1.0, float, env),
            timeline=_get("TIMELINE", "", str, env),
            stall_check_s=_get("STALL_CHECK_TIME_SECONDS", 60.0, float, env),
            stall_shutdown_s=_get("STALL_SHUTDOWN_TIME_SECONDS", 0.0, float, env),
            stall_check_disable=_get("STALL_CHECK_DISABLE", False, bool, env),
            hierarchical_allreduce=_get("HIERARCHICAL_ALLREDUCE", False, bool, env),
            adasum_flat=_get("ADASUM_FLAT", False, bool, env),
            consistency_check=_get("CONSISTENCY_CHECK", True, bool, env),
            fault=_get("FAULT", "", str, env),
            log_level=_get("LOG_LEVEL", "INFO", str, env).upper(),
            timeout_s=_get("TIMEOUT_SECONDS", 600.0, float, env),
            autotune=_get("AUTOTUNE", False, bool, env),
            autotune_candidates=_get("AUTOTUNE_CANDIDATES", "1,4,16,64", str, env),
            autotune_warmup_steps=_get("AUTOTUNE_WARMUP_STEPS", 3, int, env),
            autotune_trial_steps=_get("AUTOTUNE_TRIAL_STEPS", 8, int, env),
            autotune_log=_get("AUTOTUNE_LOG", "", str, env),
            roctx=_get("ROCTX", False, bool, env),
            negotiate=_get("NEGOTIATE", False, bool, env),
            engine=_get("ENGINE", "auto", str, env).strip().lower(),
            store=_get("STORE", "native", str, env),
            debug_sync=_get("DEBUG_SYNC", False, bool, env),
            elastic_grace_s=_get("ELASTIC_GRACE_SECONDS", 30.0, float, env),
            elastic_timeout_s=_get("ELASTIC_TIMEOUT_SECONDS", 600.0, float, env),
        )
