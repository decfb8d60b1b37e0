"""Race detection for the native runtime (SURVEY.md §5 "race detection /
sanitizers"): the C++ DynamicBatcher (csrc/runtime/batcher.cpp) is compiled
host-only with ThreadSanitizer and AddressSanitizer and driven by CPU fake
instances from many producer threads (csrc/tests/batcher_stress.cpp).  The
reference has no sanitizer story (its only thread-safety device is a
``threading.Lock`` around the ORT session cache, src/shared/model/
registry.py:128,155-159)."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SRCS = [ROOT / "csrc" / "tests" / "batcher_stress.cpp", ROOT / "csrc" / "runtime" / "batcher.cpp",
        ROOT / "csrc" / "runtime" / "trace.cpp", ROOT / "csrc" / "runtime" / "jpeg_decode.cpp"]


def _build(sanitizer: str) -> Path:
    if not (Path(HIPCC).exists() or shutil.which(HIPCC)):
        pytest.skip("hipcc not available")
    out = ROOT / "build" / f"batcher_stress_{sanitizer}"
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in SRCS + list((ROOT / "csrc" / "runtime").glob("*.h")))
    if not out.exists() or out.stat().st_mtime < newest:
        # host code only: each -fsanitize= goes right after -Xarch_host
        cmd = [HIPCC, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", f"-fsanitize={sanitizer}",
               "-I" + str(ROOT / "csrc"), *map(str, SRCS), "-ldl", "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
    return out


@pytest.mark.parametrize("sanitizer", ["thread", "address"])
def test_batcher_stress_under_sanitizer(sanitizer):
    exe = _build(sanitizer)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    assert "ThreadSanitizer" not in report and "AddressSanitizer" not in report, report[-6000:]
    assert r.returncode == 0, report[-6000:]
    assert "batcher_stress: ok" in r.stdout



@pytest.mark.parametrize("sanitizer", ["thread", "address"])
def test_string_pool_under_sanitizer(sanitizer):
    """The front end's request-body pool (csrc/runtime/string_pool.h): bodies filled on producer threads, put back
    from consumer threads, oversized ones freed, the pool bounded (csrc/tests/string_pool_stress.cpp)."""
    if not (Path(HIPCC).exists() or shutil.which(HIPCC)):
        pytest.skip("hipcc not available")
    src = ROOT / "csrc" / "tests" / "string_pool_stress.cpp"
    out = ROOT / "build" / f"string_pool_stress_{sanitizer}"
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(src.stat().st_mtime, (ROOT / "csrc" / "runtime" / "string_pool.h").stat().st_mtime)
    if not out.exists() or out.stat().st_mtime < newest:
        cmd = [HIPCC, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", f"-fsanitize={sanitizer}",
               "-I" + str(ROOT / "csrc"), str(src), "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([str(out), "5000"], capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    assert "ThreadSanitizer" not in report and "AddressSanitizer" not in report, report[-6000:]
    assert r.returncode == 0 and "string_pool_stress: ok" in r.stdout, report[-3000:]


def test_arrivals_merge_while_a_batch_is_in_flight():
    """Requests trickling in (1 per ms) while the instance is busy (10 ms of 'device' time per batch,
    EchoInstance latency_us) are merged into the next batch rather than launched one by one: the instance
    loop blocks on the oldest in-flight batch before it looks at the queue again (batcher.cpp)."""
    import threading
    import time

    import numpy as np

    from inference_arena_amd.ops import native

    C = native()
    b = C.DynamicBatcher([C.EchoInstance(4, 32, 4, 10000)], {"max_batch": 32, "max_queue_delay_us": 500})
    done = threading.Semaphore(0)
    img = np.full((8, 8, 3), 7, np.uint8)
    t0 = time.perf_counter()
    for _ in range(40):
        assert b.enqueue(img, lambda d: done.release()) >= 0
        time.sleep(0.001)
    for _ in range(40):
        assert done.acquire(timeout=10)
    elapsed = time.perf_counter() - t0
    hist = b.stats()["batch_hist"]
    b.shutdown()
    sizes = [n for n, c in enumerate(hist) for _ in range(c)]
    assert sum(sizes) == 40 and len(sizes) <= 10 and max(sizes) >= 5, sizes
    assert elapsed >= 0.01  # the simulated device time was honoured


def test_idle_queue_delay_applies_only_while_idle():
    """idle_queue_delay_us: a lone request on an idle instance waits the short idle delay, not
    max_queue_delay_us (default -1: the max delay, Triton semantics)."""
    import threading
    import time

    import numpy as np

    from inference_arena_amd.ops import native

    C = native()
    img = np.full((8, 8, 3), 7, np.uint8)

    def lone_request_s(cfg) -> float:
        b = C.DynamicBatcher([C.EchoInstance(4, 32, 4)], {"max_batch": 32, **cfg})
        done = threading.Event()
        t0 = time.perf_counter()
        assert b.enqueue(img, lambda d: done.set()) >= 0
        assert done.wait(10)
        dt = time.perf_counter() - t0
        b.shutdown()
        return dt

    assert lone_request_s({"max_queue_delay_us": 300000}) >= 0.25  # Triton semantics: waits for company
    assert lone_request_s({"max_queue_delay_us": 300000, "idle_queue_delay_us": 1000}) < 0.1


def test_overlap_admits_due_batches_while_one_runs():
    """overlap=1 (ARENA_BATCH_OVERLAP): while a batch is in flight and a slot is free, a batch that comes due is
    submitted at once instead of waiting for the oldest batch (the instance answers ready(): EchoInstance like the
    Executor); overlap=0 keeps the merge-behind-the-oldest behaviour."""
    import threading
    import time

    import numpy as np

    from inference_arena_amd.ops import native

    C = native()
    img = np.full((8, 8, 3), 7, np.uint8)

    def run(overlap):
        b = C.DynamicBatcher([C.EchoInstance(4, 8, 4, 50000)],
                             {"max_batch": 8, "max_queue_delay_us": 500, "overlap": overlap})
        done = threading.Semaphore(0)
        t0 = time.perf_counter()
        for _ in range(4):
            assert b.enqueue(img, lambda d: done.release()) >= 0
            time.sleep(0.005)
        for _ in range(4):
            assert done.acquire(timeout=10)
        elapsed = time.perf_counter() - t0
        hist = b.stats()["batch_hist"]
        b.shutdown()
        return elapsed, [n for n, c in enumerate(hist) for _ in range(c)]

    t_on, sizes_on = run(1)
    t_off, sizes_off = run(0)
    assert sizes_on == [1, 1, 1, 1], sizes_on  # four overlapping batches
    assert len(sizes_off) == 2, sizes_off     # the first alone, the rest merged behind it
    assert t_on < 0.09 and t_off >= 0.095, (t_on, t_off)
