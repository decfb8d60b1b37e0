#!/usr/bin/env python3
"""Per-layer conv microbenchmark across kernel implementations (MI355X).

Every OP_CONV of the pipeline program is replayed standalone at the bench
batch (32 images / crop capacity) with random inputs; each implementation
(ARENA conv impl 1 direct, 2 LDS tiles, 3 igemm) is timed with HIP events and
checked against impl 2's output.

    python tools/bench_convs.py --impls 2,3 --iters 20 --out gpurun_out/convs.md
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    import torch

    from inference_arena_amd.engine.planner import CROPS, OP_CONV
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import functional as AF
    from inference_arena_amd.ops import native

    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="2,3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--images", type=int, default=32)
    ap.add_argument("--crops", type=int, default=128)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ops", default=None, help="comma-separated op indices to run (default: all convs)")
    a = ap.parse_args(argv)
    C = native()
    impls = [int(i) for i in a.impls.split(",")]
    prog = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    lines = ["| op | shape | " + " | ".join(f"impl{i} us" for i in impls) + " | best | max diff |",
             "|---|---|" + "---|" * len(impls) + "---|---|"]
    tot = {i: 0.0 for i in impls}
    for k, r in enumerate(prog.ops):
        if int(r[0]) != OP_CONV or (a.ops and str(k) not in a.ops.split(",")):
            continue
        H, W, Cin, Ho, Wo, Cout, KH, KW, S, pt, pl = (int(v) for v in (r[4], r[5], r[6], r[13], r[14], r[15],
                                                                       r[17], r[18], r[19], r[20], r[21]))
        f32 = bool(r[29])
        B = a.crops if int(r[30]) == CROPS else a.images
        x = (torch.rand(B, H, W, Cin, generator=g) * 2 - 0.5).to(torch.bfloat16).to(dev)
        w = torch.randn(Cout, Cin, KH, KW, generator=g) / (Cin * KH * KW) ** 0.5
        b = torch.randn(Cout, generator=g) * 0.1
        packed = AF.pack_weights(w, b, dev)
        res = torch.rand(B, Ho, Wo, Cout, generator=g).to(torch.bfloat16).to(dev) if int(r[22]) != -1 else None
        outs, times = {}, {}
        for impl in impls:
            C.set_conv_impl(impl)
            kw = dict(stride=S, pad=(pt, pl), act="silu", out_hw=(Ho, Wo), f32out=f32, res=res, packed=packed)
            y = AF.conv2d_nhwc(x, w, b, **kw)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                AF.conv2d_nhwc(x, w, b, out=y, **kw)
            e1.record()
            torch.cuda.synchronize()
            times[impl] = e0.elapsed_time(e1) * 1e3 / a.iters
            outs[impl] = y.float()
            tot[impl] += times[impl]
        ref = outs[impls[0]]
        diff = max(float((o - ref).abs().max()) for o in outs.values())
        best = min(times, key=times.get)
        shape = f"{B}x{H}x{W}x{Cin}->{Ho}x{Wo}x{Cout} k{KH} s{S}"
        lines.append(f"| {k} | {shape} | " + " | ".join(f"{times[i]:.1f}" for i in impls) + f" | {best} | {diff:.3g} |")
    lines.append("| total | | " + " | ".join(f"{tot[i]:.0f}" for i in impls) + " | | |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
