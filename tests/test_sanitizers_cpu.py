"""Race detection / memory checking of the native host runtime.

The self-test (csrc/runtime/tests/selftest.cc) drives every multi-threaded component with real
concurrency — the TCP store server with 8 client threads and parked GETs, the negotiation engine
with 4 ranks as threads submitting reused names in different orders, the timeline writer and the
stall inspector — and is run under ThreadSanitizer and under AddressSanitizer +
UndefinedBehaviorSanitizer. Any report fails the test. GPU sanitizers (ASan/xnack) are not
available on the MI355X pool, so device code is covered by the numerics tests instead.
"""
import os
import subprocess

import pytest

from mihvd import _build

pytestmark = pytest.mark.slow


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_runtime_selftest_under_sanitizer(kind, tmp_path):
    exe = _build.build_selftest(kind)
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 exitcode=66 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1 halt_on_error=1 exitcode=66"
    env["UBSAN_OPTIONS"] = "halt_on_error=1 print_stacktrace=1"
    p = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    report = p.stdout[-4000:] + p.stderr[-8000:]
    assert p.returncode == 0, report
    assert "runtime selftest ok" in p.stdout
    for marker in ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:", "LeakSanitizer"):
        assert marker not in p.stderr, report
