"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host code: the CPU
oracle and the host build of the device physics headers (tests/sanitize/*).  Host code only -- GPU
sanitizers are not available on this pool."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "sanitize")])


@pytest.mark.parametrize("prog", ["oracle_asan", "hostcheck_asan"])
def test_sanitized_run(built, prog):
    r = subprocess.run([os.path.join(BUILD, prog)], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
