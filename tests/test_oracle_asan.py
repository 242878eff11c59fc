"""SURVEY §5 (sanitizers): the CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer.

oracle/Makefile's asan target builds lib/liboracle_asan.so with -fsanitize=address,undefined;
tests/asan/oracle_under_asan.py drives its entry points in a child process that preloads the
sanitizer runtimes (ctypes loads the library into an uninstrumented interpreter).  Any report
fails the run (halt_on_error for both)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_clean_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"])
    env = dict(os.environ, LD_PRELOAD=asan + " " + ubsan, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "asan", "oracle_under_asan.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
