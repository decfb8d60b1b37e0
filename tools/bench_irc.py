#!/usr/bin/env python3
"""Standalone timing of the fused fp32 inverted-residual kernels (csrc/kernels/ir_crop_f32.hip and
ir_f32.hip) on MobileNetV2 block shapes, over ``--crops`` crops; ``--dbg`` lists diagnostic phase masks of
ir_crop_f32 (1 no expand MFMA, 2 no depthwise, 4 no project MFMA, 8 no per-chunk weight fetch, 16 no Wp
staging store) to locate where a chunk's time goes.

Usage (GPU): python tools/bench_irc.py [--crops 128] [--dbg 0,1,2,4,8,16,31]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = [  # (H, inp, hid, oup, stride, res)
    (112, 32, 32, 16, 1, False), (112, 16, 96, 24, 2, False), (56, 24, 144, 24, 1, True),
    (56, 24, 144, 32, 2, False), (28, 32, 192, 32, 1, True), (28, 32, 192, 64, 2, False),
    (14, 64, 384, 64, 1, True), (14, 64, 384, 96, 1, False), (14, 96, 576, 96, 1, True),
    (14, 96, 576, 160, 2, False), (7, 160, 960, 160, 1, True), (7, 160, 960, 320, 1, False),
]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crops", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dbg", default="0")
    ap.add_argument("--small", action="store_true", help="also the 14x14 / 7x7 shapes (ir_crop_f32)")
    a = ap.parse_args(argv)
    import torch

    from inference_arena_amd.engine.planner import ir_crop_f32_planned, pack_ir_weights, split_bf16x3
    from inference_arena_amd.ops import native
    from inference_arena_amd.ops.functional import _ptr, _stream

    C = native()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for H, inp, hid, oup, s, res in SHAPES:
        x = torch.randn(a.crops, H, H, inp, generator=g).to(dev)
        expand = None if hid == inp else (torch.randn(hid, inp, 1, 1, generator=g) / inp ** 0.5,
                                          torch.randn(hid, generator=g) * 0.1)
        dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
        proj = (torch.randn(oup, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(oup, generator=g) * 0.1)
        pk = pack_ir_weights(expand, dw, proj, inp, k_align=16)
        Ho = (H - 1) // s + 1
        y = torch.empty(a.crops, Ho, Ho, oup, device=dev)
        x3 = ir_crop_f32_planned(H, s, pk["inp_pad"], pk["hid_pad"], pk["oup_pad"], int(expand is not None))
        if H <= 14 and not a.small:
            continue
        w = {k: pk[k].float().contiguous().to(dev) for k in ("we", "be", "wd", "bd", "wp", "bp")}
        if x3:
            w["we"], w["wp"] = split_bf16x3(pk["we"]).to(dev), split_bf16x3(pk["wp"]).to(dev)
        for dbg in ([int(v) for v in a.dbg.split(",")] if x3 else [0]):
            d = {"x": _ptr(x), "x_cs": inp, "H": H, "W": H, "inp": inp, "inp_pad": pk["inp_pad"],
                 "hid_pad": pk["hid_pad"], "oup": oup, "oup_pad": pk["oup_pad"], "stride": s,
                 "expand": int(expand is not None),
                 "res": int(res), **{k: _ptr(v) for k, v in w.items()}, "y": _ptr(y), "y_cs": oup, "Ho": Ho,
                 "Wo": Ho, "B": a.crops, "bdev": 0, "stream": _stream(), "f32": 1, "x3w": int(x3) | (dbg << 4)}
            for _ in range(3):
                C.ir_block(d)
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.reps):
                C.ir_block(d)
            t1.record()
            torch.cuda.synchronize()
            print(json.dumps({"H": H, "inp": inp, "hid": hid, "oup": oup, "s": s, "x3": bool(x3), "dbg": dbg,
                              "us": round(t0.elapsed_time(t1) / a.reps * 1e3, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
