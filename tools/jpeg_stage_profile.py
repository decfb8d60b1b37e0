#!/usr/bin/env python3
"""Per-batch cost of the split decoder's device half from a rocprofv3 run of
``tools/profile_engine.py --inputs jpeg`` (``--kernel-trace --memory-copy-trace``): the JPEG reconstruction
kernels (dequantisation + islow IDCT, chroma upsampling + colour conversion; csrc/kernels/jpeg_idct.hip) and the
host -> device copies of each batch (the coefficient blocks DMA'd from pinned memory plus the control block).
Batches are delimited by the program's first kernel (stamp_kernel)."""
from __future__ import annotations

import argparse
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def _rows(path: Path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", help="rocprofv3 output directory (searched recursively)")
    ap.add_argument("--skip", type=int, default=3, help="warm-up batches to drop")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    d = Path(a.dir)
    kt = next(iter(sorted(d.rglob("*kernel_trace.csv"))), None)
    mt = next(iter(sorted(d.rglob("*memory_copy_trace.csv"))), None)
    if kt is None:
        print("no kernel trace under", d, file=sys.stderr)
        return 1
    ks = sorted(_rows(kt), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in ks if "stamp_kernel" in r["Kernel_Name"]]
    # every program has 3 stamps (start, classifier start, end): a batch begins at every third
    starts = starts[::3]
    per = defaultdict(lambda: defaultdict(float))
    names = set()

    def batch_of(t):
        # the reconstruction of batch b runs just before its program's first stamp
        for i, s in enumerate(starts):
            if t < s:
                return i
        return len(starts)

    for r in ks:
        n = r["Kernel_Name"]
        if "jpeg" not in n:
            continue
        import re

        m = re.search(r"(jpeg_\w+)", n)
        short = m.group(1) if m else n
        names.add(short)
        per[batch_of(int(r["Start_Timestamp"]))][short] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    copies = defaultdict(lambda: [0, 0.0, 0])
    if mt is not None:
        for r in _rows(mt):
            direction = (r.get("Direction") or r.get("Operation") or r.get("Kind") or "")
            if "HOST_TO_DEVICE" not in direction.upper() and "H2D" not in direction.upper():
                continue
            b = batch_of(int(r["Start_Timestamp"]))
            size = int(r.get("Size") or r.get("Bytes") or r.get("Copy_Bytes") or 0)
            c = copies[b]
            c[0] += size
            c[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            c[2] += 1
    batches = sorted(b for b in per if b >= a.skip and b < len(starts))
    lines = ["| stage | mean us / batch | min | max |", "|---|---|---|---|"]
    for n in sorted(names):
        v = [per[b][n] for b in batches]
        lines.append(f"| {n} | {statistics.mean(v):.1f} | {min(v):.1f} | {max(v):.1f} |")
    if copies:
        cb = [b for b in batches if b in copies]
        if cb:
            lines.append(f"| H2D copies (count {statistics.mean(copies[b][2] for b in cb):.0f}) | "
                         f"{statistics.mean(copies[b][1] for b in cb):.1f} | - | - |")
            mb = statistics.mean(copies[b][0] for b in cb) / 1e6
            us = statistics.mean(copies[b][1] for b in cb)
            lines.append(f"| H2D MB / batch | {mb:.2f} ({mb / max(us, 1e-9) * 1e-6 * 1e6:.1f} GB/s over the copy time) | - | - |")
    lines.append("")
    lines.append(f"{len(batches)} batches (after {a.skip} warm-up); trace {kt.name}" + (f", {mt.name}" if mt else ""))
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
