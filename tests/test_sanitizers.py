"""CPU: AddressSanitizer / UndefinedBehaviorSanitizer / ThreadSanitizer runs of the host code
(SURVEY.md §5 promised them; the reference itself builds -O2 -DNDEBUG with none, and has
unsynchronised Shard-thread writes).

* oracle/ (the C restatement, the literal reference loop, the GMP decode and the threaded
  TF-Shard-like baseline) under ASan+UBSan, cross-checking each other on seeded specials,
  random bit patterns and random / malformed hex text;
* the threaded baseline under TSan (1, 4 and 7 threads over a ragged split);
* libefl_hip.so's host side (fxp.hip's C-ABI argument checks and error text, version.cpp) built
  with `-Xarch_host -fsanitize=address,undefined` and driven through every invalid-argument path
  without a GPU.

Builds go to tools/sanitize/build (tools/sanitize/Makefile)."""
import os
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "tools", "sanitize")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-j3", "-C", SAN])
    return os.path.join(SAN, "build")


def _run(exe, *args, env=None):
    e = dict(os.environ, **(env or {}))
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
    return r.stdout


def test_oracle_asan_ubsan(built):
    assert "ok" in _run(os.path.join(built, "oracle_asan"),
                        env={"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1"})


def test_threaded_baseline_tsan(built):
    assert "ok" in _run(os.path.join(built, "oracle_tsan"), "threads", env={"TSAN_OPTIONS": "halt_on_error=1"})


def test_abi_host_side_asan_ubsan(built):
    # leak detection off: the HIP runtime keeps process-lifetime allocations
    assert "ok" in _run(os.path.join(built, "abi_asan"),
                        env={"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1"})
