#!/usr/bin/env python3
"""A/B of the fp32 stride-1 inverted-residual kernels on the MobileNetV2 56x56 / 28x28 block shapes over
``--crops`` crops: the register-resident kernel (csrc/kernels/ir_reg_x3.hip) against the tiled one
(ir_tile_x3.hip), same split-plane weights, plus the max error of each against an fp64 torch reference.

Usage (GPU): python tools/bench_irreg.py [--crops 128] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = [(56, 24, 144, 24, 1, True), (28, 32, 192, 32, 1, True)]  # (H, inp, hid, oup, stride, res)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crops", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args(argv)
    import torch
    import torch.nn.functional as F

    from inference_arena_amd.ops import functional as AF
    from inference_arena_amd.ops import native

    C = native()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for H, inp, hid, oup, s, res in SHAPES:
        x = torch.randn(a.crops, H, H, inp, generator=g)
        expand = (torch.randn(hid, inp, 1, 1, generator=g) / inp ** 0.5, torch.randn(hid, generator=g) * 0.1)
        dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
        proj = (torch.randn(oup, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(oup, generator=g) * 0.1)
        xd = x.to(dev)
        k = min(8, a.crops)
        xc = x[:k].permute(0, 3, 1, 2).double()
        hh = F.conv2d(xc, expand[0].double(), expand[1].double()).clamp(0, 6)
        hh = F.conv2d(hh, dw[0].double(), dw[1].double(), stride=s, padding=1, groups=hid).clamp(0, 6)
        ref = F.conv2d(hh, proj[0].double(), proj[1].double()) + (xc if res else 0)
        for name, on in (("reg", 1), ("tile", 0)):
            C.set_ir_reg(on)
            y = AF.ir_block_nhwc(xd, expand, dw, proj, stride=s, res=res)
            err = (y[:k].permute(0, 3, 1, 2).double().cpu() - ref).abs().max().item()
            for _ in range(2):
                AF.ir_block_nhwc(xd, expand, dw, proj, stride=s, res=res)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # time the kernel alone: ir_block_nhwc re-packs weights per call, so time a captured call sequence
            ts = []
            for _ in range(a.reps):
                t0.record()
                AF.ir_block_nhwc(xd, expand, dw, proj, stride=s, res=res)
                t1.record()
                torch.cuda.synchronize()
                ts.append(t0.elapsed_time(t1))
            ts.sort()
            print(json.dumps({"H": H, "inp": inp, "hid": hid, "oup": oup, "kernel": name, "crops": a.crops,
                              "us_p50_with_pack": round(ts[len(ts) // 2] * 1e3, 1), "max_err": err}), flush=True)
        C.set_ir_reg(-1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
