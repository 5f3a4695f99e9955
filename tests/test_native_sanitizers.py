"""Race / memory-error detection for the native runtime (the
reference runs TSAN/ASAN builds of its C++ in CI). Builds
csrc/runtime/{object_store,channel}.cc together with the stress driver
csrc/runtime/tests/stress_runtime.cc under ThreadSanitizer and under
AddressSanitizer+UBSan (host code only), runs the multi-thread / multi-process
stress, and requires a clean report. A deliberately racy canary build must be
flagged, so a silently non-instrumented build cannot pass."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")
SRCS = [os.path.join(RT, "tests", "stress_runtime.cc"), os.path.join(RT, "object_store.cc"),
        os.path.join(RT, "channel.cc")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build(tmp_path, sanitize, extra=()):
    out = str(tmp_path / ("stress_" + sanitize.replace(",", "_")))
    cmd = ["g++", "-O1", "-g", "-std=c++17", f"-fsanitize={sanitize}", "-fno-omit-frame-pointer",
           "-I", RT, *extra, *SRCS, "-o", out, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _run(binary, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([binary, *map(str, args)], capture_output=True, text=True, timeout=600, env=e)


def test_threadsanitizer_clean(tmp_path):
    b = _build(tmp_path, "thread")
    r = _run(b, 4, 1500, env={"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "stress_runtime rc=0" in r.stdout


def test_address_undefined_sanitizer_clean(tmp_path):
    b = _build(tmp_path, "address,undefined")
    r = _run(b, 4, 1500, env={"ASAN_OPTIONS": "detect_leaks=1 halt_on_error=1",
                              "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1"})
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "stress_runtime rc=0" in r.stdout


def test_threadsanitizer_canary_is_flagged(tmp_path):
    b = _build(tmp_path, "thread", extra=("-DSTRESS_CANARY_RACE",))
    r = _run(b, env={"TSAN_OPTIONS": "halt_on_error=0"})
    assert "WARNING: ThreadSanitizer: data race" in r.stderr
