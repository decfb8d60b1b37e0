"""Native crash tracer (csrc/runtime/crash_trace.cpp): a fault on a thread Python's faulthandler cannot name
still prints the native stack, and the process still dies by the signal (the previous handler runs after it)."""
import os
import signal
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

_PROG = """
import sys, threading, ctypes
sys.path.insert(0, {root!r})
from inference_arena_amd.ops import native
C = native()
print("installed", C.crash_trace_installed(), flush=True)
t = threading.Thread(target=lambda: ctypes.string_at(8))
t.start(); t.join()
"""


def _run(env_extra):
    env = dict(os.environ, ARENA_AUTOBUILD="0", **env_extra)
    return subprocess.run([sys.executable, "-c", _PROG.format(root=str(ROOT))], capture_output=True, text=True,
                          env=env, timeout=120, cwd="/tmp")


@pytest.mark.parametrize("faulthandler", ["0", "1"])
def test_native_thread_fault_prints_native_stack(faulthandler):
    env = {"ARENA_CRASH_TRACE": "1"}
    if faulthandler == "1":
        env["PYTHONFAULTHANDLER"] = "1"
    r = _run(env)
    if "installed" not in r.stdout:
        pytest.skip(f"native extension not importable: {r.stderr[-400:]}")
    assert "installed True" in r.stdout
    assert r.returncode in (-signal.SIGSEGV, 128 + signal.SIGSEGV), r.returncode
    assert "[arena crash] fatal signal 11 (SIGSEGV) on native thread" in r.stderr
    assert "fault address 0x8" in r.stderr
    assert "libc.so" in r.stderr and "[arena crash]   #0 " in r.stderr
    if faulthandler == "1":  # chained: faulthandler still reports the Python threads
        assert "Fatal Python error: Segmentation fault" in r.stderr


def test_crash_trace_can_be_disabled():
    r = _run({"ARENA_CRASH_TRACE": "0"})
    if "installed" not in r.stdout:
        pytest.skip(f"native extension not importable: {r.stderr[-400:]}")
    assert "installed False" in r.stdout
    assert "[arena crash]" not in r.stderr
    assert r.returncode in (-signal.SIGSEGV, 128 + signal.SIGSEGV)
