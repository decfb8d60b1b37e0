#!/usr/bin/env python3
"""Per-thread CPU of this process in phases (which threads burn CPU while the serving path idles or waits).

Phases, each sampled for --secs seconds from /proc/self/task/*/stat (utime + stime):
  torch    after ``import torch`` (no device touched)
  device   after the first HIP call (torch.cuda.init + one tiny kernel)
  engine   after building the fused pipeline and running one batch, idle
  loaded   while a thread keeps batches of --batch images in flight through the native batcher
Each thread's name, CPU % and current syscall (/proc/<tid>/syscall: a number = blocked in that call, "running" =
user space) is printed for threads above 1 %.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
HZ = os.sysconf("SC_CLK_TCK")


def _threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{tid}/stat").read()
        except OSError:
            continue
        l, r = st.find("("), st.rfind(")")
        f = st[r + 2:].split()
        out[int(tid)] = (st[l + 1:r], int(f[11]) + int(f[12]))
    return out


def _syscall(tid):
    try:
        s = open(f"/proc/self/task/{tid}/syscall").read().split()
        return s[0] if s else "?"
    except OSError:
        return "?"


def phase(name, secs, dump=0):
    a = _threads()
    t0 = time.monotonic()
    time.sleep(secs)
    dt = time.monotonic() - t0
    b = _threads()
    rows = []
    for tid, (nm, tk) in b.items():
        pct = 100.0 * (tk - a.get(tid, (nm, tk))[1]) / HZ / dt
        rows.append((pct, tid, nm, _syscall(tid)))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"== {name}: {len(rows)} threads, {tot:.1f} % CPU", flush=True)
    for pct, tid, nm, sc in rows:
        if pct >= 1.0:
            print(f"   {nm:16s} tid {tid:7d} {pct:6.1f} %  syscall {sc}", flush=True)
    if dump:  # native stacks of the busiest threads, a few samples each (stderr)
        from inference_arena_amd.ops import native

        for pct, tid, nm, sc in rows[:dump]:
            for _ in range(3):
                native().dump_thread_stack(tid)
                time.sleep(0.05)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dump", type=int, default=0, help="native stacks of the N busiest threads per phase")
    a = ap.parse_args(argv)
    import torch

    phase("torch", a.secs)
    torch.cuda.init()
    x = torch.ones(16, device="cuda")
    (x * 2).sum().item()
    phase("device", a.secs)
    import numpy as np

    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.registry import build_session
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import native

    yolo, mnet = default_models(0)
    pipe = build_session("pipeline", yolo, mnet, device=0, buckets=[1, a.batch])
    imgs = synthetic_images(a.batch, 3)
    pipe.infer(imgs)
    phase("engine", a.secs)
    stop_r = threading.Event()

    n_rep = [0]

    def replay():  # graph launches only (+ one stream sync per 20): is the runtime's event thread busy here too?
        while not stop_r.is_set():
            n_rep[0] += 20
            pipe.ex.replay(a.batch, 0, 20)
            pipe.ex.synchronize()

    tr = threading.Thread(target=replay, daemon=True)
    tr.start()
    time.sleep(0.3)
    r0, t0 = n_rep[0], time.perf_counter()
    phase("replay", a.secs, dump=a.dump)
    print(f"   replay rate {(n_rep[0] - r0) / (time.perf_counter() - t0):.0f} graphs/s", flush=True)
    stop_r.set()
    tr.join(10)
    C = native()
    b = C.DynamicBatcher([pipe.ex], {"max_batch": a.batch, "max_queue_delay_us": 200})
    stop = threading.Event()
    frames = [np.ascontiguousarray(i) for i in imgs]

    def drive():
        import queue

        q: queue.Queue = queue.Queue()
        while not stop.is_set():
            for i, f in enumerate(frames):
                b.enqueue(f, lambda r: q.put(1))
            for _ in frames:
                q.get()

    t = threading.Thread(target=drive, daemon=True)
    t.start()
    time.sleep(0.5)
    phase("loaded", a.secs, dump=a.dump)
    stop.set()
    t.join(10)
    b.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
