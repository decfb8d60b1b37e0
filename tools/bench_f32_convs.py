#!/usr/bin/env python3
"""fp32 conv tile-variant sweep (MI355X).

Every OP_CONV of the fp32 pipeline program is replayed standalone at the bench
batch (32 images / 128 crops) with random fp32 inputs.  Each is timed under the
default dispatch policy (impl 0), every explicit LDS implicit-GEMM tile
variant (impl 10 + v, the table in csrc/kernels/conv_f32.hip
``launch_lds_variant``) the fp32-accurate triple-bf16-split variants (impl 40 + v) and the 3x3 halo
kernel (impl 100, where eligible); the
outputs are checked against the direct kernel (impl 1).  The result table is
what the dispatch policy of ``conv2d_f32`` is set from.

    python tools/bench_f32_convs.py --iters 20 --out gpurun_out/f32_variants.md
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

VARIANTS = {  # v: (BM, BN, KC) as instantiated in launch_lds_variant
    0: (64, 64, 32), 1: (128, 64, 32), 2: (64, 128, 32), 3: (128, 128, 32), 4: (64, 64, 64),
    5: (128, 64, 64), 6: (64, 128, 64), 7: (128, 32, 32), 8: (256, 16, 32), 9: (128, 48, 32),
    10: (128, 80, 32), 11: (64, 64, 32), 12: (128, 64, 32), 13: (32, 64, 32), 14: (128, 32, 64),
    15: (128, 48, 64),
}


def main(argv=None) -> int:
    import torch

    from inference_arena_amd.engine.planner import CROPS, OP_CONV
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import functional as AF
    from inference_arena_amd.ops import native

    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--images", type=int, default=32)
    ap.add_argument("--crops", type=int, default=128)
    ap.add_argument("--variants", default=",".join(str(v) for v in VARIANTS))
    ap.add_argument("--x3", default=",".join(str(v) for v in range(12)),
                    help="triple-bf16-split variants (impl 40 + v); empty = none")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    C = native()
    variants = [int(v) for v in a.variants.split(",") if v != ""]
    prog = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype="fp32")
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    x3 = [int(v) for v in a.x3.split(",") if v != ""]
    cols = ["default"] + [f"v{v}" for v in variants] + [f"x{v}" for v in x3] + ["halo", "xhalo"] + \
        [f"g{v}" for v in range(6)]
    lines = ["| op | shape | " + " | ".join(cols) + " | best | gain us | max rel err fp32 | max rel err x3 |",
             "|---|---|" + "---|" * len(cols) + "---|---|---|---|"]
    tot_default = tot_best = 0.0
    for k, r in enumerate(prog.ops):
        if int(r[0]) != OP_CONV:
            continue
        H, W, Cin, Ho, Wo, Cout, KH, KW, S, pt, pl = (int(v) for v in (r[4], r[5], r[6], r[13], r[14], r[15],
                                                                       r[17], r[18], r[19], r[20], r[21]))
        B = a.crops if int(r[30]) == CROPS else a.images
        x = (torch.rand(B, H, W, Cin, generator=g) * 2 - 0.5).to(dev)
        w = torch.randn(Cout, Cin, KH, KW, generator=g) / (Cin * KH * KW) ** 0.5
        b = torch.randn(Cout, generator=g) * 0.1
        packed = AF.pack_weights(w, b, dev, "fp32")
        res = torch.rand(B, Ho, Wo, Cout, generator=g).to(dev) if int(r[22]) != -1 else None
        base = dict(stride=S, pad=(pt, pl), act="silu", out_hw=(Ho, Wo), res=res, packed=packed)
        ref = torch.empty(B, Ho, Wo, Cout, device=dev)
        try:
            _conv(C, AF, x, packed, ref, 1, base, KH, KW, Cout, res)  # direct kernel = reference
        except RuntimeError as e:
            print(f"| {k} | skipped: {e} |", flush=True)
            continue
        times, errs = {}, {}
        impls = ([("default", 0)] + [(f"v{v}", 10 + v) for v in variants] + [(f"x{v}", 40 + v) for v in x3] +
                 [("halo", 100), ("xhalo", 101)] + [(f"g{v}", 111 + v) for v in range(6)])
        for name, impl in impls:
            y = torch.empty_like(ref)

            def run():
                _conv(C, AF, x, packed, y, impl, base, KH, KW, Cout, res)
            try:
                run()
                torch.cuda.synchronize()
            except RuntimeError:
                continue
            errs[name] = float((y - ref).abs().max() / ref.abs().max().clamp_min(1e-6))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[name] = e0.elapsed_time(e1) * 1e3 / a.iters
        best = min(times, key=times.get)
        tot_default += times["default"]
        tot_best += times[best]
        shape = f"{B}x{H}x{W}x{Cin}->{Ho}x{Wo}x{Cout} k{KH} s{S}"
        cells = [f"{times[c]:.1f}" if c in times else "-" for c in cols]
        lines.append(f"| {k} | {shape} | " + " | ".join(cells) +
                     f" | {best} | {times['default'] - times[best]:.1f} | "
                     f"{max([e for n, e in errs.items() if not n.startswith('x')], default=0):.2e} | "
                     f"{max([e for n, e in errs.items() if n.startswith('x')], default=0):.2e} |")
        print(lines[-1], flush=True)
    lines.append(f"| total | | default {tot_default:.0f} us, best-of {tot_best:.0f} us |")
    lines.append("")
    lines.append("max rel err = max |y - y_direct| / max |y_direct| over all implementations of the op (the direct "
                 "exact-fp32 kernel is the reference; x* are the triple-bf16-split kernels)")
    text = "\n".join(lines)
    print(lines[-1])
    if a.out:
        Path(a.out).write_text(text + "\n")
    return 0


def _conv(C, AF, x, packed, y, impl, base, KH, KW, Cout, res):
    """conv2d_f32 with an explicit ConvParams.impl (bypasses the global policy)."""
    wt, bt, kpad, cpad, w3 = packed
    B, H, W, Cx = x.shape
    Ho, Wo = base["out_hw"]
    pt, pl = base["pad"]
    C.conv2d({
        "x": x.data_ptr(), "B": B, "H": H, "W": W, "xs": Cx, "Cin": Cx,
        "w": wt.data_ptr(), "Kpad": kpad, "bias": bt.data_ptr(),
        "y": y.data_ptr(), "Ho": Ho, "Wo": Wo, "ys": Cout, "Cout": Cout, "Cout_pad": cpad,
        "KH": KH, "KW": KW, "stride": base["stride"], "pad_t": pt, "pad_l": pl,
        "res": res.data_ptr() if res is not None else 0, "rs": Cout if res is not None else 0,
        "y2": 0, "y2s": 0, "act": AF.ACT["silu"], "f32out": 0, "bdev": 0,
        "stream": AF._stream(), "f32": 1, "impl": impl, "w3": w3.data_ptr(),
    })


if __name__ == "__main__":
    raise SystemExit(main())
