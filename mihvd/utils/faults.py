"""Fault injection driven by ``MIHVD_FAULT``, parsed by the native ``FaultPlan``.

Spec: ``kind:key=val:...;kind2:...`` with kinds ``kill`` (exit with ``code``, default 1),
``delay`` (sleep ``ms``), ``hang`` (sleep ``s``, default 3600 — the stall inspector must catch it),
``raise`` (RuntimeError), ``nan`` (returns True so the caller poisons a gradient) and ``collerr``
(a communicator async error of ``code``, default 6 = remote error, reported to the native health
monitor, which aborts the communicator and exits with 134 like a real RCCL failure).
``rank=`` and ``step=`` select where it fires (absent = everywhere / every step).
"""
from __future__ import annotations

import os
import sys
import time

from .. import basics


def maybe_inject(step: int) -> bool:
    """Apply every fault due at ``step`` on this rank. Returns True if a ``nan`` fault fired."""
    plan = basics._ctx.fault_plan
    if plan is None:
        return False
    nan = False
    for a in plan.due(basics.rank(), int(step)):
        if a.kind == "kill":
            print(f"[rank {basics.rank()}] MIHVD_FAULT: kill at step {step}", file=sys.stderr, flush=True)
            os._exit(int(a.args.get("code", "1")))
        elif a.kind == "delay":
            time.sleep(float(a.args.get("ms", "100")) / 1000.0)
        elif a.kind == "hang":
            time.sleep(float(a.args.get("s", "3600")))
        elif a.kind == "raise":
            raise RuntimeError(f"MIHVD_FAULT: injected failure at step {step}")
        elif a.kind == "nan":
            nan = True
        elif a.kind == "collerr":
            mon = basics._ctx.health
            if mon is None:
                raise RuntimeError("MIHVD_FAULT collerr needs the health monitor (MIHVD_HEALTH=1)")
            mon.inject_error(int(a.args.get("code", "6")), f"MIHVD_FAULT at step {step}")
            time.sleep(float(a.args.get("s", "30")))  # the monitor exits the process meanwhile
    return nan
