"""Lowering of the two oracle networks into one executor program.

The whole request pipeline of the reference's monolithic arm
(architectures/monolithic/app/inference.py:127-227: decode -> letterbox ->
YOLO -> NMS -> un-letterbox -> per-detection crop -> MobileNet -> argmax) is
lowered into a single device-resident program:

  letterbox(s2d) -> 75 YOLOv5nu convs (+SPPF pool) -> decode -> NMS ->
  crop plan -> crop gather(s2d) -> 52 MobileNetV2 convs/dwconvs -> avgpool ->
  FC -> top-5

Lowering rules (what replaces ONNX graph nodes):
  * BN is folded into every conv; SiLU / ReLU6 / residual Add are epilogues.
  * Concat nodes disappear: producers store into channel slices of a shared
    buffer; the two FPN Upsample nodes become the conv epilogue's second,
    2x-nearest store (h10 and h14 feed both a concat at their own resolution
    and an upsampled concat).
  * C3's cv1 and cv2 (same input) are one conv with stacked weights; the
    bottleneck chain updates the cv1 half in place.
  * Detect's first 3x3 convs of the box and class branches are one conv.
  * Both stems read space-to-depth inputs: YOLO's 6x6/s2/p2 conv becomes a
    3x3/s1 conv over 12(+4) channels, MobileNet's 3x3/s2 conv a 2x2/s1 conv.
  * With ``ARENA_FUSE_STEM`` (default) the letterbox / crop gather is fused
    into those stem convs (stem_fused op): the s2d input only exists in LDS.

Precision (``dtype``): ``"bf16"`` lowers onto the tuned bf16 kernels and every
fusion above; ``"fp32"`` lowers onto the exact-fp32 kernels (fp32 activations
and weights, fp32 MFMA; csrc/kernels/conv_f32.hip) with the unfused op set —
the reference's numerics (ONNX Runtime fp32, reference experiment.yaml:202-225).
"""
from __future__ import annotations

import os

import torch

from ..models.common import fold, fold_conv_bn
from ..models.mobilenetv2 import MobileNetV2
from ..models.yolov5nu import STRIDES, YOLOv5nu
from .planner import BUF_NONE, BUF_RAWOUT, BUF_XCROPS, CROPS, IMAGES, Program, ProgramBuilder, Reserved, View

CAND_BYTES = 32
CROPREF_BYTES = 32


def s2d_stem_6x6(w: torch.Tensor) -> torch.Tensor:
    """[Co,3,6,6] (stride 2, pad 2) -> [Co,16,3,3] (stride 1, pad 1) over space-to-depth input."""
    co = w.shape[0]
    out = torch.zeros(co, 16, 3, 3)
    for a in range(3):
        for b in range(3):
            for p in range(2):
                for q in range(2):
                    for c in range(3):
                        out[:, (p * 2 + q) * 3 + c, a, b] = w[:, c, 2 * a + p, 2 * b + q]
    return out


def s2d_stem_3x3(w: torch.Tensor) -> torch.Tensor:
    """[Co,3,3,3] (stride 2, pad 1) -> [Co,16,2,2] (stride 1, pad top/left 1) over space-to-depth input."""
    co = w.shape[0]
    out = torch.zeros(co, 16, 2, 2)
    tap = {(0, 1): 0, (1, 0): 1, (1, 1): 2}  # (block offset a, phase p) -> original tap i
    for (a, p), i in tap.items():
        for (b, q), j in tap.items():
            for c in range(3):
                out[:, (p * 2 + q) * 3 + c, a, b] = w[:, c, i, j]
    return out


# (C1, c_, bottlenecks, shortcut) combinations csrc/kernels/c3_fused.hip implements (YOLOv5n's 160x160 and
# 80x80 C3 blocks); H % 8 == 0 and W % 16 == 0 are also required.
C3_FUSED = {(32, 16, 1, True), (64, 32, 2, True), (128, 32, 1, False)}
# Where the fused kernel measured faster on MI355X (batch 32, serial kernel trace): the 160x160 block
# (c_ = 16: 56 us vs 90 us for its four convs).  At 80x80 (c_ = 32) the fused kernels are LDS-occupancy
# bound (69-75 KB per workgroup) and only break even (b4) or lose (h17), so they stay unfused by default.
C3_FUSED_AUTO = {(32, 16, 1, True)}


def fuse_c3_policy() -> str:
    """``ARENA_FUSE_C3``: ``auto`` (default, measured-faster shapes only), ``all`` or ``none``/``0``."""
    v = os.environ.get("ARENA_FUSE_C3", "auto").lower()
    return {"0": "none", "false": "none", "off": "none", "1": "auto", "true": "auto"}.get(v, v)


def fuse_c3_f32() -> bool:
    """``ARENA_FUSE_C3_F32`` (default 1): fp32 programs run the 160x160 C3 block (C1 32, c_ 16, one bottleneck) as
    one fp32-accurate kernel (csrc/kernels/c3_x3.hip) instead of four convs (101.7 vs 156 us per batch of 32,
    profiles/r4h/)."""
    return os.environ.get("ARENA_FUSE_C3_F32", "1").lower() not in ("0", "false", "no", "off")


def _c3(pb: ProgramBuilder, m, src: View, dst: View, H: int, W: int, name: str) -> None:
    c_ = m.c_
    res = bool(m.m[0].add)
    if pb.f32:
        allowed = {(32, 16, 1, True)} if fuse_c3_f32() and fuse_c3_policy() != "none" else set()
    else:
        policy = fuse_c3_policy()
        allowed = C3_FUSED if policy == "all" else C3_FUSED_AUTO if policy == "auto" else set()
    if ((src.C, c_, len(m.m), res) in allowed and H % 8 == 0 and W % 16 == 0
            and all(bool(bn.add) == res for bn in m.m)):
        w1, b1 = fold(m.cv1)
        w2, b2 = fold(m.cv2)
        pb.c3_fused(src, dst, H, W, (torch.cat([w1, w2]), torch.cat([b1, b2])),
                    [(fold(bn.cv1), fold(bn.cv2)) for bn in m.m], fold(m.cv3), res=res)
        return
    T = pb.tensor(f"{name}.T", H, W, 2 * c_)
    U = pb.tensor(f"{name}.U", H, W, c_)
    w1, b1 = fold(m.cv1)
    w2, b2 = fold(m.cv2)
    pb.conv(src, View(T, 0, 2 * c_), torch.cat([w1, w2]), torch.cat([b1, b2]))
    for bn in m.m:
        wa, ba = fold(bn.cv1)
        pb.conv(View(T, 0, c_), View(U, 0, c_), wa, ba)
        wb, bb = fold(bn.cv2)
        pb.conv(View(U, 0, c_), View(T, 0, c_), wb, bb, res=View(T, 0, c_) if bn.add else None)
    w3, b3 = fold(m.cv3)
    pb.conv(View(T, 0, 2 * c_), dst, w3, b3)


def fuse_stem_default() -> bool:
    """``ARENA_FUSE_STEM`` (default 1): preprocessing fused into the stem convs (stem_fused op)."""
    return os.environ.get("ARENA_FUSE_STEM", "1").lower() not in ("0", "false", "no", "off")


def fuse_stem2_default() -> bool:
    """``ARENA_FUSE_STEM2`` (default 1): with the fused stem, the detector's second conv (3x3 s2,
    16 -> 32) runs in the same kernel; the 320x320x16 stem output is never stored."""
    return os.environ.get("ARENA_FUSE_STEM2", "1").lower() not in ("0", "false", "no", "off")


def fuse_stem_ir_default() -> bool:
    """``ARENA_FUSE_STEM_IR`` (default 1): with the fused stem, MobileNetV2's first inverted residual
    (t = 1) runs in the same kernel; the 112x112x32 stem output is never stored."""
    return os.environ.get("ARENA_FUSE_STEM_IR", "1").lower() not in ("0", "false", "no", "off")


def fuse_head_pool_default() -> bool:
    """``ARENA_FUSE_POOL`` (default 1): MobileNetV2's last 1x1 conv and the global average pool run as one
    kernel (head_pool op); the 7x7x1280 map is never stored."""
    return os.environ.get("ARENA_FUSE_POOL", "1").lower() not in ("0", "false", "no", "off")


def fuse_letterbox_f32_default() -> bool:
    """``ARENA_F32_LB_STEM`` (default 1): in fp32 programs the stem conv samples the letterboxed images
    itself (letterbox_conv); the 320x320x16 fp32 space-to-depth input is never stored."""
    return os.environ.get("ARENA_F32_LB_STEM", "1").lower() not in ("0", "false", "no", "off")


def fuse_stem_s2_f32_default() -> bool:
    """``ARENA_F32_STEM_S2`` (default 1): fp32 programs run letterbox + stem + the 3x3 s2 conv as one kernel
    (csrc/kernels/stem_x3.hip): the 320x320x16 fp32 stem map exists only in LDS.  0 keeps the letterbox-sampling
    stem conv + a separate s2 conv (A/B switch)."""
    return os.environ.get("ARENA_F32_STEM_S2", "1").lower() not in ("0", "false", "no", "off")


def plan_yolo(pb: ProgramBuilder, y: YOLOv5nu, T: int = 640, tensor_input: bool = False,
              fuse_stem: bool | None = None):
    h = T // 2
    w, b = fold(y.b0)
    if fuse_stem is None:
        fuse_stem = fuse_stem_default()
    # fp32: only the letterbox + stem + s2 conv form exists (csrc/kernels/stem_x3.hip, ARENA_F32_STEM_S2)
    fuse_stem = fuse_stem and (not pb.f32 or fuse_stem_s2_f32_default())
    A1 = pb.tensor("b1", h // 2, h // 2, 32)
    if fuse_stem and not tensor_input and (fuse_stem2_default() or pb.f32) and T % 64 == 0:
        # letterbox + stem + b1 (3x3 s2) in one kernel: the 320x320x16 stem output stays in LDS
        w1, b1 = fold(y.b1)
        pb.stem_fused(View(A1, 0, 32), s2d_stem_6x6(w), b, S=T, act="silu", second=(w1, b1, "silu"))
    elif fuse_stem and not tensor_input and not pb.f32:
        A0 = pb.tensor("b0", h, h, 16)
        pb.stem_fused(View(A0, 0, 16), s2d_stem_6x6(w), b, S=T, act="silu")
        pb.conv(View(A0, 0, 16), View(A1, 0, 32), *fold(y.b1), stride=2)
    elif pb.f32 and not tensor_input and fuse_letterbox_f32_default():
        A0 = pb.tensor("b0", h, h, 16)
        pb.letterbox_conv(View(A0, 0, 16), s2d_stem_6x6(w), b, T=T)
        pb.conv(View(A0, 0, 16), View(A1, 0, 32), *fold(y.b1), stride=2)
    else:
        A0 = pb.tensor("b0", h, h, 16)
        X0 = pb.tensor("x_s2d", h, h, 16)
        if tensor_input:
            pb.tensor_in(X0, T)
        else:
            pb.letterbox(X0, T)
        pb.conv(View(X0, 0, 16), View(A0, 0, 16), s2d_stem_6x6(w), b)
        pb.conv(View(A0, 0, 16), View(A1, 0, 32), *fold(y.b1), stride=2)
    A2 = pb.tensor("b2", h // 2, h // 2, 32)
    _c3(pb, y.b2, View(A1, 0, 32), View(A2, 0, 32), h // 2, h // 2, "b2")
    s8 = T // 8
    A3 = pb.tensor("b3", s8, s8, 64)
    pb.conv(View(A2, 0, 32), View(A3, 0, 64), *fold(y.b3), stride=2)
    CAT16 = pb.tensor("cat16", s8, s8, 128)
    _c3(pb, y.b4, View(A3, 0, 64), View(CAT16, 64, 64), s8, s8, "b4")
    s16 = T // 16
    A5 = pb.tensor("b5", s16, s16, 128)
    pb.conv(View(CAT16, 64, 64), View(A5, 0, 128), *fold(y.b5), stride=2, src_hw=(s8, s8))
    CAT12 = pb.tensor("cat12", s16, s16, 256)
    _c3(pb, y.b6, View(A5, 0, 128), View(CAT12, 128, 128), s16, s16, "b6")
    s32 = T // 32
    A7 = pb.tensor("b7", s32, s32, 256)
    pb.conv(View(CAT12, 128, 128), View(A7, 0, 256), *fold(y.b7), stride=2)
    A8 = pb.tensor("b8", s32, s32, 256)
    _c3(pb, y.b8, View(A7, 0, 256), View(A8, 0, 256), s32, s32, "b8")
    S9 = pb.tensor("sppf", s32, s32, 512)
    c_ = y.b9.c_
    pb.conv(View(A8, 0, 256), View(S9, 0, c_), *fold(y.b9.cv1))
    pb.sppf(S9, c_)
    A9 = pb.tensor("b9", s32, s32, 256)
    pb.conv(View(S9, 0, 4 * c_), View(A9, 0, 256), *fold(y.b9.cv2))
    CAT22 = pb.tensor("cat22", s32, s32, 256)
    pb.conv(View(A9, 0, 256), View(CAT22, 128, 128), *fold(y.h10), dst2=View(CAT12, 0, 128))
    A13 = pb.tensor("h13", s16, s16, 128)
    _c3(pb, y.h13, View(CAT12, 0, 256), View(A13, 0, 128), s16, s16, "h13")
    CAT19 = pb.tensor("cat19", s16, s16, 128)
    pb.conv(View(A13, 0, 128), View(CAT19, 64, 64), *fold(y.h14), dst2=View(CAT16, 0, 64))
    P3 = pb.tensor("p3", s8, s8, 64)
    _c3(pb, y.h17, View(CAT16, 0, 128), View(P3, 0, 64), s8, s8, "h17")
    pb.conv(View(P3, 0, 64), View(CAT19, 0, 64), *fold(y.h18), stride=2)
    P4 = pb.tensor("p4", s16, s16, 128)
    _c3(pb, y.h20, View(CAT19, 0, 128), View(P4, 0, 128), s16, s16, "h20")
    pb.conv(View(P4, 0, 128), View(CAT22, 0, 128), *fold(y.h21), stride=2)
    P5 = pb.tensor("p5", s32, s32, 256)
    _c3(pb, y.h23, View(CAT22, 0, 256), View(P5, 0, 256), s32, s32, "h23")

    d = y.detect
    c2, c3, nc = d.c2, d.c3, d.nc
    # bf16: the v3 halo-tile kernel's epilogue; fp32: the x3hg epilogue variants (csrc/kernels/halo_x3g.hip)
    fuse_head = os.environ.get("ARENA_FUSE_HEAD", "1").lower() not in ("0", "false", "no", "off")
    ch = c2 + c3
    heads = []
    lanes = head_lanes()
    region = pb.parallel()
    lane = region.__enter__()
    for lvl, (P, cin, s) in enumerate(((P3, 64, s8), (P4, 128, s16), (P5, 256, s32))):
        lane(lvl + 1 if lanes else 0)  # the three levels are independent: one side stream each
        H1 = pb.tensor(f"det{lvl}.h1", s, s, ch)
        H2 = pb.tensor(f"det{lvl}.h2", s, s, ch)
        D = pb.tensor(f"det{lvl}.out", s, s, 4 * d.reg_max + nc)
        wa, ba = fold(d.cv2[lvl][0])
        wc, bc = fold(d.cv3[lvl][0])
        pb.conv(View(P, 0, cin), View(H1, 0, ch), torch.cat([wa, wc]), torch.cat([ba, bc]))
        # fp32 at 20x20: the fused x3hg tiles (8 x 16 px) would pad the map to 24 x 32, the unfused pair is
        # faster there (profiles/r3c_x3hg_ops.md ops 58-59: 33.6 + 48.0 us fused vs 18.7 + 9.6 + 27.0 + 9.9)
        if fuse_head and c2 in (64, 80) and c3 in (64, 80) and (not pb.f32 or s >= 40):
            # second 3x3 of each branch with its final 1x1 in the epilogue: the 3x3 output never leaves LDS
            pb.conv(View(H1, 0, c2), View(BUF_NONE, 0, c2), *fold(d.cv2[lvl][1]),
                    pw=(*fold_conv_bn(d.cv2[lvl][2], None), View(D, 0, 4 * d.reg_max), None))
            pb.conv(View(H1, c2, c3), View(BUF_NONE, 0, c3), *fold(d.cv3[lvl][1]),
                    pw=(*fold_conv_bn(d.cv3[lvl][2], None), View(D, 4 * d.reg_max, nc), None))
        else:
            pb.conv(View(H1, 0, c2), View(H2, 0, c2), *fold(d.cv2[lvl][1]))
            pb.conv(View(H1, c2, c3), View(H2, c2, c3), *fold(d.cv3[lvl][1]))
            pb.conv(View(H2, 0, c2), View(D, 0, 4 * d.reg_max), *fold_conv_bn(d.cv2[lvl][2], None), act=None)
            pb.conv(View(H2, c2, c3), View(D, 4 * d.reg_max, nc), *fold_conv_bn(d.cv3[lvl][2], None), act=None)
        heads.append(View(D, 0, 4 * d.reg_max + nc))
    region.__exit__(None, None, None)
    return heads


def head_lanes() -> bool:
    """``ARENA_HEAD_LANES`` (default 0): the Detect head's three levels run as parallel branches of the batch's
    graph (side streams, ProgramBuilder.parallel) in buckets up to ``ARENA_LANES_MAX_BATCH`` (2; the executor
    keeps larger buckets on one stream: with four slots in flight the side streams only add contention,
    profiles/r4lanes/); their small-grid convs (15-50 workgroups each at bs 1) leave most CUs idle when
    serialised.  The executor captures each lane run as a linear graph and launches the lanes on the slot's side
    streams (a single forked-branch graph segfaulted inside hipGraphLaunch under the arm-B services' 2-queue cap:
    profiles/r5lanes/README.md).  Off by default: bs-1 / bs-2 latency is unchanged within noise (1.907 vs 1.904 ms,
    1.992 vs 1.972 ms) and arm B at 10 users is 2 % slower with it (profiles/r5lanes/)."""
    return os.environ.get("ARENA_HEAD_LANES", "0").lower() not in ("0", "false", "no", "off")


def fuse_ir_default() -> str:
    """Inverted-residual fusion policy (``ARENA_FUSE_IR``): ``auto`` (default), ``all`` or ``none``/``0``."""
    v = os.environ.get("ARENA_FUSE_IR", "auto").lower()
    return {"0": "none", "1": "all", "false": "none", "true": "all"}.get(v, v)


def ir_crop_default() -> bool:
    """``ARENA_IR_CROP`` (default 1): MobileNetV2 blocks with a 7x7 output map and <= 160 (or 320) output channels
    run fused as one workgroup per crop (the native side reads the same variable)."""
    return os.environ.get("ARENA_IR_CROP", "1").lower() not in ("0", "false", "no", "off")


def fuse_block_f32(blk, H: int) -> bool:
    """fp32 policy: fuse the memory-bound blocks at >= 28x28 input (csrc/kernels/ir_f32.hip), where the
    unfused fp32 expanded map (up to 4.8 MB per crop) round-trips HBM, and the 14x14 / 7x7 blocks the
    whole-map triple-bf16-split kernel covers when enabled (csrc/kernels/ir_crop_f32.hip, ``ARENA_IRC_F32``); the
    rest run as batched 1x1 GEMMs + depthwise."""
    from .planner import ir_crop_f32_planned
    from .validate import ir_f32_supported

    inp_pad = (blk.inp + 15) // 16 * 16
    hid_pad = inp_pad if blk.expand is None else (blk.hidden + 31) // 32 * 32
    oup_pad = (blk.oup + 15) // 16 * 16
    expand = int(blk.expand is not None)
    if H >= 28:
        return ir_f32_supported(blk.stride, inp_pad, hid_pad, oup_pad, expand)
    return ir_crop_f32_planned(H, blk.stride, inp_pad, hid_pad, oup_pad, expand)


def irx_slices() -> int:
    """``ARENA_IRX_SLICES`` (default 6): fp32 14x14 stride-1 blocks (MobileNetV2 features[8..13]; with
    ``ARENA_IRX_TAIL`` also 14 -> 7 and 7x7) split their hidden channels over up to this many workgroups per row
    band and hand the next block partial sums (csrc/kernels/ir_crop_f32.hip, IrParams.x_parts / y_parts; the
    executor uses all of them for small crop capacities, ``ARENA_IRX_SLICES_BIG`` for full batches); 1 keeps one
    workgroup per band and plain tensors."""
    try:
        return max(1, min(8, int(os.environ.get("ARENA_IRX_SLICES", "6"))))
    except ValueError:
        return 6


def _sliceable_f32(blk, H: int) -> bool:
    """A block the hidden-sliced whole-map kernel takes: a 14x14 or 7x7 input the kernel is planned for (stride-1
    14x14 blocks; with ``ARENA_IRX_TAIL`` also 14 -> 7 and 7x7), expanding, with at least as many 32-channel
    hidden chunks as slices (the kernel's partial-sum geometry)."""
    from .planner import ir_crop_f32_planned

    if H not in (14, 7) or blk.expand is None or blk.inp % 4 or blk.oup % 4:
        return False
    inp_pad = (blk.inp + 15) // 16 * 16
    hid_pad = (blk.hidden + 31) // 32 * 32
    oup_pad = (blk.oup + 15) // 16 * 16
    return hid_pad // 32 >= irx_slices() and ir_crop_f32_planned(H, blk.stride, inp_pad, hid_pad, oup_pad, 1)


def fuse_stem_ir_f32_default() -> bool:
    """``ARENA_F32_STEM_IR`` (default 1): fp32 programs run crop gather + stem conv + MobileNetV2 block 1 as one
    kernel (ProgramBuilder.ir_block_stem); the s2d crops and the 112 x 112 x 32 stem map are never stored."""
    return os.environ.get("ARENA_F32_STEM_IR", "1").lower() not in ("0", "false", "no", "off")


def fuse_block(blk, H: int, policy) -> bool:
    if policy == "f32":
        return fuse_block_f32(blk, H)
    """``auto``: fuse where the tile kernel wins on MI355X — blocks at >= 28x28 input and the stride-1
    14x14 blocks (hid 576: 46 us fused vs 28 + 18 + 17 us as expand / depthwise / project ops;
    profiles/r1_irpolicy14_ops.md).  The 14 -> 7 stride-2 block and the 7x7 blocks have one
    output tile per crop and a 18-30 chunk serial loop in the tile kernel: unless the whole-crop
    kernel takes them (``ARENA_IR_CROP``, default 1: csrc/kernels/ir_crop.hip, waves split the hidden
    channels; <= 160 or 320 output channels) they run as batched 1x1 GEMMs + depthwise over all crops."""
    if policy in (True, "all"):
        return True
    if policy in (False, None, "none"):
        return False
    if H >= 28 or (H >= 14 and blk.stride == 1):
        return True
    Ho = (H + 2 - 3) // blk.stride + 1
    return ir_crop_default() and Ho == 7 and blk.expand is not None and (blk.oup <= 160 or blk.oup == 320)


def plan_mobilenet(pb: ProgramBuilder, m: MobileNetV2, crops, S: int, mean, std, *, kind: int = CROPS,
                   raw_logits: bool = False, fuse_ir: bool | str | None = None, fuse_stem: bool | None = None):
    """MobileNetV2 over crop-gathered inputs (``crops`` = CropRef buffer) or, with
    ``crops=None``, over fp32 [3,S,S] tensors of the image batch (``kind=IMAGES``).

    ``fuse_ir``: each inverted-residual block is one fused kernel (expand ->
    depthwise -> project, intermediates in LDS) instead of three ops with the
    expanded tensor round-tripping through HBM."""
    CROPS_ = kind
    if fuse_ir is None:
        fuse_ir = fuse_ir_default()
    h = S // 2
    if fuse_stem is None:
        fuse_stem = fuse_stem_default()
    if pb.f32:  # fp32: the fused stem is bf16-only; blocks fuse by the fp32 policy (fuse_block_f32)
        fuse_stem = False
        fuse_ir = "f32" if fuse_ir in ("auto", True, "all", "f32") else "none"
    w, b = fold(m.stem)
    b0 = m.blocks[0]
    first_fused = (fuse_stem and crops is not None and fuse_stem_ir_default() and S % 32 == 0
                   and b0.expand is None and b0.stride == 1 and not b0.use_res and b0.inp == 32 and b0.oup == 16
                   and fuse_block(b0, h, fuse_ir))
    first_fused_f32 = (pb.f32 and crops is not None and fuse_stem_ir_f32_default() and S % 2 == 0
                       and b0.expand is None and b0.stride == 1 and not b0.use_res and b0.inp == 32
                       and b0.oup <= 16 and h >= 16)
    if first_fused:
        # crop gather + stem + block 1 in one kernel: the 112x112x32 stem output stays in LDS
        O0 = pb.tensor("m0.out", h, h, b0.oup, kind=CROPS_)
        pb.stem_fused(View(O0, 0, b0.oup), s2d_stem_3x3(w), b, S=S, act="relu6", crops=crops, mean=mean, std=std,
                      kind=CROPS_, ir=(fold(b0.dw), fold(b0.project)))
        F = O0
    elif first_fused_f32:
        # fp32: crop gather + s2d stem conv + block 1 in one kernel (csrc/kernels/ir_f32.hip, IrParams.stem)
        O0 = pb.tensor("m0.out", h, h, b0.oup, kind=CROPS_)
        pb.ir_block_stem(crops, View(O0, 0, b0.oup), (s2d_stem_3x3(w), b), fold(b0.dw), fold(b0.project), S=S,
                         mean=mean, std=std, kind=CROPS_)
        F = O0
        first_fused = True
    elif fuse_stem and crops is not None:
        F = pb.tensor("m.stem", h, h, 32, kind=CROPS_)
        pb.stem_fused(View(F, 0, 32), s2d_stem_3x3(w), b, S=S, act="relu6", crops=crops, mean=mean, std=std,
                      kind=CROPS_)
    else:
        F = pb.tensor("m.stem", h, h, 32, kind=CROPS_)
        X = pb.tensor("crop_s2d", h, h, 16, kind=CROPS_)
        if crops is None:
            pb.tensor_in(X, S)
        else:
            pb.crop_gather(crops, X, S, mean, std)
        pb.conv(View(X, 0, 16), View(F, 0, 32), s2d_stem_3x3(w), b, pad=(1, 1), act="relu6", kind=CROPS_,
                out_hw=(h, h))
    cur, H = F, h
    parts = 1  # partial sums held by `cur` (hidden-sliced 14x14 blocks)
    slices = irx_slices() if pb.f32 and fuse_ir == "f32" else 1
    for i, blk in enumerate(m.blocks):
        if i == 0 and first_fused:
            continue
        Ho = (H + 2 - 3) // blk.stride + 1
        if fuse_block(blk, H, fuse_ir):
            nxt = m.blocks[i + 1] if i + 1 < len(m.blocks) else None
            yp = slices if (slices > 1 and _sliceable_f32(blk, H) and nxt is not None
                            and fuse_block(nxt, Ho, fuse_ir) and _sliceable_f32(nxt, Ho)) else 1
            O = pb.tensor(f"m{i}.out", Ho, Ho, blk.oup * yp, kind=CROPS_)
            pb.ir_block(View(cur, 0, blk.inp * parts), View(O, 0, blk.oup * yp),
                        fold(blk.expand) if blk.expand is not None else None, fold(blk.dw), fold(blk.project),
                        stride=blk.stride, res=blk.use_res, kind=CROPS_, x_parts=parts, y_parts=yp)
            cur, H, parts = O, Ho, yp
            continue
        if parts != 1:
            raise AssertionError("partial-sum tensor feeds an unfused block")
        if blk.expand is not None:
            E = pb.tensor(f"m{i}.exp", H, H, blk.hidden, kind=CROPS_)
            pb.conv(View(cur, 0, blk.inp), View(E, 0, blk.hidden), *fold(blk.expand), act="relu6", kind=CROPS_)
        else:
            E = cur
        Dw = pb.tensor(f"m{i}.dw", Ho, Ho, blk.hidden, kind=CROPS_)
        wd, bd = fold(blk.dw)
        pb.dwconv(View(E, 0, blk.hidden), View(Dw, 0, blk.hidden), wd, bd, stride=blk.stride, kind=CROPS_)
        O = pb.tensor(f"m{i}.out", Ho, Ho, blk.oup, kind=CROPS_)
        pb.conv(View(Dw, 0, blk.hidden), View(O, 0, blk.oup), *fold(blk.project), act=None,
                res=View(cur, 0, blk.inp) if blk.use_res else None, kind=CROPS_)
        cur, H = O, Ho
    PO = pb.tensor("m.pool", 1, 1, 1280, kind=CROPS_)
    if fuse_head_pool_default() and H * H <= 64 and cur.C == 320:
        pb.head_pool(View(cur, 0, cur.C), View(PO, 0, 1280), *fold(m.head), act="relu6", kind=CROPS_)
    else:
        HD = pb.tensor("m.head", H, H, 1280, kind=CROPS_)
        pb.conv(View(cur, 0, cur.C), View(HD, 0, 1280), *fold(m.head), act="relu6", kind=CROPS_)
        pb.avgpool(HD, PO, kind=CROPS_)
    ncls = m.fc.out_features
    wfc = m.fc.weight.detach().float().cpu().reshape(ncls, 1280, 1, 1)
    if raw_logits:  # reference contract: [1000] fp32 logits per input, straight into the output region
        pb.conv(View(PO, 0, 1280), View(BUF_RAWOUT, 0, ncls), wfc, m.fc.bias.detach().float().cpu(), act=None,
                f32out=True, kind=CROPS_, raw_cs=ncls)
        return
    LG = pb.tensor("m.logits", 1, 1, ncls + (-ncls % 8), kind=CROPS_, elem=4)
    pb.conv(View(PO, 0, 1280), View(LG, 0, ncls), wfc, m.fc.bias.detach().float().cpu(), act=None, f32out=True,
            kind=CROPS_)
    pb.topk(LG, ncls, LG.C)


def plan_pipeline(yolo: YOLOv5nu, mnet: MobileNetV2, *, conf_thr: float, iou_thr: float, det_size: int = 640,
                  cls_size: int = 224, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                  cand_cap: int = 8400, max_det: int = 300, dtype: str = "bf16") -> Program:
    pb = ProgramBuilder(dtype)
    pb.stamp(0)  # device wall-clock stamps: detection = [0, 1), classification = [1, 2) (reference timing keys)
    heads = plan_yolo(pb, yolo, det_size)
    cand = pb.raw("cand", cand_cap * CAND_BYTES)
    count = pb.raw("cand_count", 4)
    pb.zero(count)
    pb.decode(heads, STRIDES, cand, count, conf_thr)
    pb.nms(cand, count, iou_thr)
    crops = pb.raw("crops", max_det * CROPREF_BYTES, pinned=True)
    pb.crop_plan(crops)
    pb.begin_classifier()
    pb.stamp(1)
    plan_mobilenet(pb, mnet, crops, cls_size, mean, std)
    pb.stamp(2)
    return pb.build({"kind": "pipeline", "conf_thr": conf_thr, "iou_thr": iou_thr, "det_size": det_size, "cls_size": cls_size,
                     "cand_cap": cand_cap, "max_det": max_det})


__all__ = ["plan_pipeline", "plan_detector", "plan_classifier", "plan_yolo_raw", "plan_mobilenet_raw", "plan_yolo", "plan_mobilenet", "s2d_stem_6x6", "s2d_stem_3x3", "BUF_NONE", "IMAGES"]


def plan_detector(yolo: YOLOv5nu, *, conf_thr: float, iou_thr: float, det_size: int = 640, cand_cap: int = 8400,
                  max_det: int = 300, dtype: str = "bf16") -> Program:
    """Detection only (microservices detection service): detections per image."""
    pb = ProgramBuilder(dtype)
    heads = plan_yolo(pb, yolo, det_size)
    cand = pb.raw("cand", cand_cap * CAND_BYTES)
    count = pb.raw("cand_count", 4)
    pb.zero(count)
    pb.decode(heads, STRIDES, cand, count, conf_thr)
    pb.nms(cand, count, iou_thr)
    return pb.build({"kind": "detector", "conf_thr": conf_thr, "iou_thr": iou_thr, "det_size": det_size,
                     "cand_cap": cand_cap, "max_det": max_det})


def plan_classifier(mnet: MobileNetV2, *, cls_size: int = 224, mean=(0.485, 0.456, 0.406),
                    std=(0.229, 0.224, 0.225), max_det: int = 300, dtype: str = "bf16") -> Program:
    """Classification only (microservices classification service): every input image is one crop."""
    pb = ProgramBuilder(dtype)
    crops = pb.raw("crops", max_det * CROPREF_BYTES, pinned=True)
    pb.crop_plan(crops, whole=True)
    pb.begin_classifier()
    plan_mobilenet(pb, mnet, crops, cls_size, mean, std)
    return pb.build({"kind": "classifier", "cls_size": cls_size, "max_det": max_det})


def plan_split_detector(yolo: YOLOv5nu, *, conf_thr: float, iou_thr: float, det_size: int = 640,
                        cand_cap: int = 8400, max_det: int = 300, dtype: str = "bf16") -> Program:
    """First stage of the split topology (GPU i): detection + crop plan exported in BUF_XCROPS, which the
    classifier stage on GPU j pulls over xGMI (csrc/runtime/split.h)."""
    pb = ProgramBuilder(dtype)
    heads = plan_yolo(pb, yolo, det_size)
    cand = pb.raw("cand", cand_cap * CAND_BYTES)
    count = pb.raw("cand_count", 4)
    pb.zero(count)
    pb.decode(heads, STRIDES, cand, count, conf_thr)
    pb.nms(cand, count, iou_thr)
    pb.crop_plan(Reserved(BUF_XCROPS))
    return pb.build({"kind": "split_detector", "conf_thr": conf_thr, "iou_thr": iou_thr, "det_size": det_size,
                     "cand_cap": cand_cap, "max_det": max_det})


def plan_split_classifier(mnet: MobileNetV2, *, cls_size: int = 224, mean=(0.485, 0.456, 0.406),
                          std=(0.229, 0.224, 0.225), max_det: int = 300, dtype: str = "bf16") -> Program:
    """Second stage of the split topology (GPU j): crop gather from the peer-copied images with the peer's
    crop plan (BUF_XCROPS) -> MobileNetV2 -> top-5; the whole program is the classification pass."""
    pb = ProgramBuilder(dtype)
    pb.begin_classifier()
    plan_mobilenet(pb, mnet, Reserved(BUF_XCROPS), cls_size, mean, std)
    return pb.build({"kind": "split_classifier", "cls_size": cls_size, "max_det": max_det})


def plan_yolo_raw(yolo: YOLOv5nu, *, det_size: int = 640, dtype: str = "bf16") -> Program:
    """Reference tensor contract of model 'yolov5n': fp32 [3,640,640] -> fp32 [84, 8400]."""
    pb = ProgramBuilder(dtype)
    heads = plan_yolo(pb, yolo, det_size, tensor_input=True)
    pb.yolo_raw(heads, STRIDES)
    A = sum((det_size // s) ** 2 for s in STRIDES)
    return pb.build({"kind": "yolo_raw", "det_size": det_size, "raw_out_bytes": 84 * A * 4,
                     "output_shape": [84, A]})


def plan_mobilenet_raw(mnet: MobileNetV2, *, cls_size: int = 224, dtype: str = "bf16") -> Program:
    """Reference tensor contract of model 'mobilenetv2': fp32 [3,224,224] -> fp32 [1000]."""
    pb = ProgramBuilder(dtype)
    plan_mobilenet(pb, mnet, None, cls_size, None, None, kind=IMAGES, raw_logits=True)
    n = mnet.fc.out_features
    return pb.build({"kind": "mobilenet_raw", "cls_size": cls_size, "raw_out_bytes": n * 4, "output_shape": [n]})
