#!/usr/bin/env python3
"""Standalone timing of fp32 conv kernels on chosen layer shapes (for rocprofv3 counter passes).

    python tools/bench_x3g.py --impls 111,115,40 --shapes det_s2,c3_1x1 --iters 50

Shapes are layers of the fp32 pipeline at the bench batch (32 images / 128 crops); every impl is checked
against the exact-fp32 direct kernel (impl 1) before it is timed.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = {  # name: (B, H, Cin, Cout, k, stride)
    "det_s2_32": (32, 160, 32, 64, 3, 2),
    "det_s2_64": (32, 80, 64, 128, 3, 2),
    "det_s2_128": (32, 40, 128, 256, 3, 2),
    "c3_1x1_128": (32, 40, 128, 128, 1, 1),
    "c3_1x1_256": (32, 20, 256, 256, 1, 1),
    "neck_1x1_512": (32, 20, 512, 256, 1, 1),
    "mb_expand": (192, 7, 160, 960, 1, 1),
    "mb_project": (192, 7, 960, 320, 1, 1),
    "head_3x3": (32, 80, 64, 64, 3, 1),
    "head_144": (32, 80, 64, 144, 3, 1),
    "head_80": (32, 80, 80, 80, 3, 1),
    "c3_3x3_32": (32, 80, 32, 32, 3, 1),
    "c3_3x3_64": (32, 40, 64, 64, 3, 1),
    "c3_3x3_128": (32, 20, 128, 128, 3, 1),
    "head_144_40": (32, 40, 128, 144, 3, 1),
    "stem_16": (32, 160, 16, 16, 3, 1),
    "stem_s2": (32, 320, 16, 32, 3, 2),
    "head_144_20": (32, 20, 256, 144, 3, 1),
    "head_64_20": (32, 20, 64, 64, 3, 1),
    "head_80_20": (32, 20, 80, 80, 3, 1),
    "det_s2_128_40": (32, 40, 128, 128, 3, 2),
    "det_s2_64_80": (32, 80, 64, 64, 3, 2),
}


def main(argv=None) -> int:
    import torch

    from inference_arena_amd.ops import functional as AF

    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="111,112,113,114,115,116")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for name in a.shapes.split(","):
        B, H, Cin, Cout, k, s = SHAPES[name]
        x = (torch.rand(B, H, H, Cin, generator=g) * 2 - 0.5).to(dev)
        w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
        b = torch.randn(Cout, generator=g) * 0.1
        packed = AF.pack_weights(w, b, dev, "fp32")
        ref = AF.conv2d_nhwc(x, w, b, stride=s, act="silu", packed=packed, impl=1)
        Ho = ref.shape[1]
        flops = 2.0 * B * Ho * Ho * Cout * Cin * k * k
        cells = []
        for impl in (int(v) for v in a.impls.split(",")):
            try:
                y = AF.conv2d_nhwc(x, w, b, stride=s, act="silu", packed=packed, impl=impl)
                torch.cuda.synchronize()
            except RuntimeError:
                cells.append(f"{impl}: -")
                continue
            err = float((y - ref).abs().max() / ref.abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                AF.conv2d_nhwc(x, w, b, stride=s, act="silu", packed=packed, impl=impl, out=y)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            cells.append(f"{impl}: {us:.1f} us ({flops * 6 / us / 1e6:.0f} TF x3-eq, err {err:.1e})")
        print(f"{name} {B}x{H}x{H}x{Cin}->{Ho}x{Ho}x{Cout} k{k} s{s} | " + " | ".join(cells), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
