"""Static program builder for the native executor.

The reference hands each model to ONNX Runtime, which plans memory and
kernels internally (src/shared/model/registry.py:194-224; ORT's
``enable_mem_pattern=False`` is set there).  Here the planning is explicit:

* a *program* is a list of fixed-size int64 op records (layouts below) that
  name arena buffers by id; ``csrc/runtime/executor.cpp`` resolves them to
  device pointers per batch bucket and captures them into a hipGraph;
* buffers are NHWC tensors (or raw byte regions) sized per batch item and
  scaled by the bucket's image count or crop capacity;
* ``layout()`` assigns arena offsets by lifetime (first/last op that touches a
  buffer), so dead activations are reused and the working set of a whole
  batch stays in the MI355X's 256 MiB Infinity Cache where possible;
* weights (BN folded, kernel layouts, bf16) are packed into one blob.

Op record layouts (index: field) — keep in sync with executor.cpp:
  CONV   1 x_buf 2 x_coff 3 x_cs 4 H 5 W 6 Cin 7 w_off 8 Kpad 9 b_off 10 y_buf
         11 y_coff 12 y_cs 13 Ho 14 Wo 15 Cout 16 Cout_pad 17 KH 18 KW 19 stride
         20 pad_t 21 pad_l 22 res_buf 23 res_coff 24 res_cs 25 y2_buf 26 y2_coff
         27 y2_cs 28 act 29 f32out 30 batch_kind
         31 pw_w_off 32 pw_kpad 33 pw_b_off 34 pw_cout (0 = none) 35 pw_cout_pad 36 pw_y_buf 37 pw_y_coff
         38 pw_y_cs 39 pw_act   (pointwise conv fused into the 3x3 epilogue; y_buf may then be BUF_NONE)
         40 w3_off 41 has_w3 (fp32: weights pre-split into bf16 planes, pack_conv_weight_x3)
  DWCONV 1 x_buf 2 x_coff 3 x_cs 4 H 5 W 6 C 7 w_off 8 b_off 9 y_buf 10 y_coff
         11 y_cs 12 Ho 13 Wo 14 stride 15 act 16 batch_kind
  SPPF   1 buf 2 coff 3 cs 4 H 5 W 6 C 7 batch_kind
  LETTERBOX 1 out_buf 2 T
  ZERO   1 buf 2 bytes_per_item 3 batch_kind
  DECODE 1-4 / 5-8 / 9-12 (buf, coff, cs, hw) per level, 13-15 strides,
         16 cand_buf 17 count_buf 18 conf_thr (float bits)
  NMS    1 cand_buf 2 count_buf 3 det_buf 4 detcount_buf 5 iou_thr (float bits)
  CROPPLAN 1 det_buf 2 detcount_buf 3 crops_buf 4 whole (1: each image is one crop)
  CROPGATHER 1 crops_buf 2 out_buf 3 S 4-6 mean 7-9 inv_std (float bits)
  AVGPOOL 1 x_buf 2 HW 3 C 4 y_buf 5 batch_kind
  TOPK   1 logits_buf 2 N 3 ld 4 out_buf
  TENSORIN 1 out_buf 2 S   (fp32 [3,S,S] pool tensors -> space-to-depth bf16)
  YOLORAW  1-12 heads as DECODE, 13-15 strides, 16 out_buf (raw [84, A] fp32 per image)
  IRBLOCK  1 x_buf 2 x_coff 3 x_cs 4 H 5 W 6 inp 7 inp_pad 8 hid_pad 9 oup 10 oup_pad 11 stride
           12 expand 13 res 14 we 15 be 16 wd 17 bd 18 wp 19 bp 20 y_buf 21 y_coff 22 y_cs 23 Ho 24 Wo
           25 batch_kind 26 x3w 27 x_parts 28 y_parts (0 / 1: plain tensors; > 1: partial sums of a
           hidden-sliced 14x14 block, IrParams.x_parts) 29-30 reserved (0) 31 stem 32 crops_buf 33 S 34-36 mean
           37-39 inv_std (float bits) 40 stem w_off 41 stem b_off
           (fused MobileNetV2 inverted residual, csrc/kernels/ir_block.hip / ir_f32.hip; stem = 1: fp32 crop
            gather + s2d stem conv computed inside the block-1 kernel, x_buf unused)
  STEMFUSED 1 src (0 letterbox, 1 crop gather) 2 y_buf 3 y_coff 4 y_cs 5 S 6 w_off 7 Kpad 8 b_off
           9 Cout 10 act 11 crops_buf 12-14 mean 15-17 inv_std (float bits) 18 batch_kind 19 KS
           20 second-conv flag 21 w2_off 22 Kpad2 23 b2_off 24 Cout2 25 act2 (y = the second conv's output)
           26 first-IR-block flag 27 wd_off 28 bd_off 29 wp_off 30 bp_off 31 oup (y = the block's output)
           (preprocessing fused into the stem conv; the s2d input exists only in LDS,
            csrc/kernels/stem_fused.hip)
  C3FUSED 1 x_buf 2 x_coff 3 x_cs 4 H 5 W 6 C1 7 CH 8 NB 9 res 10 w12 11 b12 12-15 (wb1, bb1, wb2, bb2) of
           bottleneck 0, 16-19 of bottleneck 1, 20 w3 21 b3 22 y_buf 23 y_coff 24 y_cs 25 batch_kind
           (whole YOLOv5 C3 block, intermediates in LDS, csrc/kernels/c3_fused.hip)
  HEADPOOL 1 x_buf 2 x_coff 3 x_cs 4 HW 5 K 6 w_off 7 Kpad 8 b_off 9 N 10 Npad 11 y_buf 12 y_coff 13 y_cs
           14 act 15 batch_kind
           (MobileNetV2 head 1x1 conv + activation + global average pool, csrc/kernels/head_pool.hip)
  STAMP    1 index (0 program start, 1 classifier start, 2 end): the device wall clock into the results
           (per-batch detection / classification device time; executor BatchResult det_ms / cls_ms)

Every record: field 47 (``OP_DTYPE_FIELD``) = activation precision of the op, 0 = bf16 activations and
weights with fp32 accumulation (the tuned fused kernels), 1 = exact fp32 (fp32 activations and weights,
v_mfma_f32_16x16x4_f32; csrc/kernels/conv_f32.hip) — the reference's ONNX Runtime precision
(reference experiment.yaml:202,207,220,225).  fp32 programs use the unfused op set (CONV, DWCONV, SPPF,
LETTERBOX, DECODE, CROPGATHER, AVGPOOL, TENSORIN, YOLORAW + the dtype-free NMS / CROPPLAN / TOPK / ZERO);
their conv weights are fp32 [Cout_pad][Kpad] with Kpad a multiple of 16.
"""
from __future__ import annotations

import os

import struct
from dataclasses import dataclass, field

import numpy as np
import torch

OP_FIELDS = 48
OP_DTYPE_FIELD = 47
OP_LANE_FIELD = 46  # stream lane of the op (0: the batch's stream; 1-3: side streams, executor.h kLaneField)
MAX_LANES = 3
DTYPES = ("bf16", "fp32")
(OP_CONV, OP_DWCONV, OP_SPPF, OP_LETTERBOX, OP_ZERO, OP_DECODE, OP_NMS, OP_CROPPLAN, OP_CROPGATHER, OP_AVGPOOL,
 OP_TOPK, OP_TENSORIN, OP_YOLORAW, OP_IRBLOCK, OP_STEMFUSED, OP_C3FUSED, OP_HEADPOOL, OP_STAMP) = range(1, 19)
BUF_NONE, BUF_CTRL, BUF_META, BUF_POOL, BUF_DET, BUF_DETCOUNT, BUF_TOPK, BUF_RAWOUT = -1, -10, -11, -12, -13, -14, -15, -16
BUF_XCROPS = -17  # crop plan exported to a second-stage executor (split topology; executor.h)


@dataclass(frozen=True)
class Reserved:
    """A reserved (executor-owned) region used where a planner Buffer is expected."""
    id: int
IMAGES, CROPS = 0, 1
ACT = {None: 0, "none": 0, "silu": 1, "relu6": 2}
ALIGN = 256


def fbits(v: float) -> int:
    return struct.unpack("<I", struct.pack("<f", float(v)))[0]


def _round(v: int, a: int) -> int:
    return (v + a - 1) // a * a


@dataclass
class Buffer:
    id: int
    name: str
    per_item: int  # bytes per batch item
    kind: int  # IMAGES or CROPS
    H: int = 0
    W: int = 0
    C: int = 0
    elem: int = 2
    pinned: bool = False  # live until the end of the program
    first: int = 1 << 30
    last: int = -1


@dataclass
class View:
    buf: Buffer | int  # Buffer or a reserved id
    coff: int = 0
    C: int = 0

    @property
    def bid(self) -> int:
        return self.buf.id if isinstance(self.buf, Buffer) else int(self.buf)

    @property
    def cs(self) -> int:
        return self.buf.C if isinstance(self.buf, Buffer) else 0


@dataclass
class Program:
    ops: np.ndarray
    cls_ops: np.ndarray
    buffers: list[Buffer]
    weights: np.ndarray
    meta: dict = field(default_factory=dict)


class WeightPacker:
    def __init__(self) -> None:
        self.chunks: list[bytes] = []
        self.size = 0

    def add(self, data: bytes) -> int:
        off = self.size
        pad = _round(len(data), ALIGN) - len(data)
        self.chunks.append(data + b"\0" * pad)
        self.size += len(data) + pad
        return off

    def blob(self) -> np.ndarray:
        return np.frombuffer(b"".join(self.chunks), dtype=np.uint8).copy()


def bf16_bytes(t: torch.Tensor) -> bytes:
    return t.detach().float().contiguous().to(torch.bfloat16).view(torch.int16).numpy().tobytes()


def split_bf16x3(t: torch.Tensor) -> torch.Tensor:
    """fp32 [..., K] -> bf16 [..., 3, K]: planes h = rn(t), m = rn(t - h), l = rn(t - h - m) (round to nearest
    even, as v_cvt_pk_bf16_f32): h + m + l equals t to fp32 rounding.  The operand format of the
    triple-bf16-split kernels (csrc/kernels/ir_crop_f32.hip)."""
    t = t.detach().float()
    h = t.to(torch.bfloat16)
    r = t - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack([h, m, lo], dim=-2).contiguous()


def bf16_raw_bytes(t: torch.Tensor) -> bytes:
    return t.contiguous().view(torch.int16).numpy().tobytes()


def f32_bytes(t: torch.Tensor) -> bytes:
    return t.detach().float().contiguous().numpy().tobytes()


def pack_conv_weight(w: torch.Tensor, b: torch.Tensor, dtype: str = "bf16") -> tuple[bytes, bytes, int, int]:
    """[Cout, Cin, KH, KW] fp32 -> ([Cout_pad][Kpad] weight bytes, bias fp32 bytes, Kpad, Cout_pad).

    bf16: Kpad a multiple of 32 (one v_mfma_f32_16x16x32_bf16 K-step); fp32: fp32 weights, Kpad a
    multiple of 16 (four v_mfma_f32_16x16x4_f32 steps)."""
    cout, cin, kh, kw = w.shape
    k = kh * kw * cin
    kpad = _round(k, 16 if dtype == "fp32" else 32)
    cpad = _round(cout, 16)
    wk = torch.zeros(cpad, kpad, dtype=torch.float32)
    wk[:cout, :k] = w.detach().float().permute(0, 2, 3, 1).reshape(cout, k)
    bb = torch.zeros(cpad, dtype=torch.float32)
    bb[:cout] = b.detach().float()
    return (f32_bytes(wk) if dtype == "fp32" else bf16_bytes(wk)), bb.numpy().tobytes(), kpad, cpad


def pack_conv_weight_x3(w: torch.Tensor) -> bytes:
    """[Cout, Cin, KH, KW] fp32 -> the pre-split operand of the x3g / x3h kernels (csrc/kernels/gemm_x3.hip):
    K ordered (ky, kx, c) with each tap's channels zero-padded to Cin32 = ceil(Cin / 32) * 32, so that a 32-deep
    K chunk kc = tap * Cin32 / 32 + c0 / 32 is one tap's channels c0 .. c0 + 31; split into bf16 planes
    (split_bf16x3) and stored [KH * KW * Cin32 / 32][Cout_pad][h 32 | m 32 | l 32]: one chunk of consecutive
    output channels is one contiguous run of 192-byte rows."""
    cout, cin, kh, kw = w.shape
    cin32 = _round(cin, 32)
    cpad = _round(cout, 16)
    wk = torch.zeros(cpad, kh * kw, cin32, dtype=torch.float32)
    wk[:cout, :, :cin] = w.detach().float().permute(0, 2, 3, 1).reshape(cout, kh * kw, cin)
    planes = split_bf16x3(wk.reshape(cpad, kh * kw * cin32 // 32, 32))  # [cpad][kc][3][32]
    return bf16_raw_bytes(planes.permute(1, 0, 2, 3).contiguous())


def pack_pw_weight_x3(w2: torch.Tensor, k2: int) -> bytes:
    """Detect-head final 1x1 [Cout2, K, 1, 1] fp32 -> the operand of the fused x3hg epilogue
    (csrc/kernels/halo_x3g.hip, PWN > 0): rows padded to 32, split into bf16 planes, stored
    [round32(Cout2)][h | m | l][k2] with the K columns in the order the 3x3 accumulators hold the channels:
    column 16 ks + 8 h + i is channel 16 ks + 4 h + (i & 3) + 8 (i >> 2)."""
    co2, k = w2.shape[0], w2.shape[1]
    rows = _round(co2, 32)
    wk = torch.zeros(rows, k2, dtype=torch.float32)
    wk[:co2, :k] = w2.detach().float().reshape(co2, k)
    col = torch.arange(k2)
    ks, h, i = col // 16, (col % 16) // 8, col % 8
    perm = 16 * ks + 4 * h + (i & 3) + 8 * (i >> 2)
    planes = split_bf16x3(wk[:, perm])  # [rows][3][k2]
    return bf16_raw_bytes(planes.contiguous())


def pack_stem_s2_x3(w0: torch.Tensor, w1: torch.Tensor) -> tuple[bytes, bytes]:
    """fp32 detector front end (csrc/kernels/stem_x3.hip): the s2d stem weights [16, 16, 3, 3] divided by 255
    (the kernel stages the letterboxed uint8 values k) as bf16 planes [3 ky][2 slabs][16 ch][h|m|l][32 k]
    (slab k = kx * 16 + c for k < 48, zero for 48..63), and the 3x3 s2 conv [32, 16, 3, 3] as
    [9 taps][32 ch][h|m|l][16 c]."""
    w0 = w0.detach().float() / 255.0
    k = torch.zeros(16, 3, 64)
    k[:, :, :48] = w0.permute(0, 2, 3, 1).reshape(16, 3, 48)  # [n][ky][kx * 16 + c]
    p0 = split_bf16x3(k.reshape(16, 3, 2, 32))  # [n][ky][sl][3][32]
    p0 = p0.permute(1, 2, 0, 3, 4).contiguous()  # [ky][sl][n][3][32]
    w1 = w1.detach().float().permute(2, 3, 0, 1).reshape(9, 32, 16)  # [tap][n][c]
    p1 = split_bf16x3(w1)  # [tap][n][3][16]
    return bf16_raw_bytes(p0), bf16_raw_bytes(p1.contiguous())


def pack_ir_weights(expand, dw, project, inp: int, k_align: int = 32) -> dict:
    """Padded operand layouts of the fused inverted-residual kernels (csrc/kernels/ir_block.hip, ir_f32.hip):
    we [hid_pad][inp_pad], wd [9][hid_pad], wp [oup_pad][hid_pad] + fp32 biases.  ``k_align``: inp_pad
    granularity (32 for the bf16 MFMA K-step, 16 for the fp32 kernel's K-chunk)."""
    wd, bd = dw
    wp, bp = project
    hid, oup = wd.shape[0], wp.shape[0]
    inp_pad = _round(inp, k_align)
    hid_pad = inp_pad if expand is None else _round(hid, 32)
    oup_pad = _round(oup, 16)
    if expand is None and hid != inp:
        raise ValueError("ir_block without expand needs hidden == inp")
    we = torch.zeros(hid_pad, inp_pad)
    be = torch.zeros(hid_pad)
    if expand is not None:
        we[:hid, :inp] = expand[0].reshape(hid, inp)
        be[:hid] = expand[1]
    wdp = torch.zeros(9, hid_pad)
    wdp[:, :hid] = wd.reshape(hid, 9).t()
    bdp = torch.zeros(hid_pad)
    bdp[:hid] = bd
    wpp = torch.zeros(oup_pad, hid_pad)
    wpp[:oup, :hid] = wp.reshape(oup, hid)
    bpp = torch.zeros(oup_pad)
    bpp[:oup] = bp
    return {"we": we, "be": be, "wd": wdp, "bd": bdp, "wp": wpp, "bp": bpp, "inp": inp, "inp_pad": inp_pad,
            "hid_pad": hid_pad, "oup": oup, "oup_pad": oup_pad}


def ir_crop_f32_policy() -> str:
    """``ARENA_IRC_F32``: ``auto`` (default), ``all``/``1`` or ``none``/``0`` — which fp32 MobileNetV2 14x14 / 7x7
    blocks run as the fused x3 kernel (csrc/kernels/ir_crop_f32.hip).  ``auto`` takes the stride-1 14x14 blocks,
    where it measured faster than the unfused expand GEMM + depthwise + project GEMM in the pipeline (128 crops:
    hid 384 61-63 vs 77 us, hid 384 -> 96 70 vs 90 us, hid 576 106-107 vs 134 us); the 14 -> 7 block and the
    7x7 blocks stay unfused (103 vs 88, 149 vs 97, 194 vs 120 us): each of their workgroups streams the block's
    whole 1.8-2.8 MB of split weights for 21-28 output pixels (profiles/r3_irx_ops.md)."""
    v = os.environ.get("ARENA_IRC_F32", "auto").lower()
    return {"1": "all", "true": "all", "yes": "all", "on": "all", "0": "none", "false": "none", "no": "none",
            "off": "none"}.get(v, v)


def ir_crop_f32_enabled() -> bool:
    return ir_crop_f32_policy() != "none"


def ir_tile_x3_enabled() -> bool:
    """``ARENA_IR_X3T`` (default 1): fp32 programs run the expanding MobileNetV2 blocks of the >= 28x28 stages on
    the tiled x3 kernel (csrc/kernels/ir_tile_x3.hip, split-plane weights) instead of the exact-fp32 ir_f32
    kernel; 0 restores ir_f32 (A/B switch)."""
    return os.environ.get("ARENA_IR_X3T", "1").lower() not in ("0", "false", "no", "off")


def stem_x3_enabled() -> bool:
    """``ARENA_STEM_X3`` (default 1): the fp32 classifier front end (crop gather + stem conv + block 1) runs its
    two GEMMs as x3 MFMAs (csrc/kernels/ir_tile_x3.hip ir_stem_x3_kernel); 0 keeps ir_f32.hip's exact-fp32
    stem mode (A/B switch)."""
    return os.environ.get("ARENA_STEM_X3", "1").lower() not in ("0", "false", "no", "off")


def ir_x3_plan(H: int, W: int, stride: int, inp: int, hid_pad: int, oup_pad: int, expand: int) -> tuple[int, int]:
    """fp32 block -> (x3w, inp_pad): 1 with the 32-aligned input padding of the x3 kernels when the whole-map
    (14x14 / 7x7) or the tiled x3 kernel takes the block, else (0, the exact-fp32 16-aligned padding)."""
    from .validate import ir_tile_x3_supported

    inp16, inp32 = _round(inp, 16), _round(inp, 32)
    if H == W and ir_crop_f32_planned(H, stride, inp16, hid_pad, oup_pad, expand):
        return 1, inp16
    # an input that would be half zero padding in the 32-deep x3 K step (MobileNetV2 block 2, 16 channels)
    # stays on ir_f32: 238 vs 215 us per batch of 32 requests (profiles/r3_fp32_itx_ops.md)
    if ir_tile_x3_enabled() and inp16 == inp32 and ir_tile_x3_supported(stride, inp32, hid_pad, oup_pad, expand):
        return 1, inp32
    return 0, inp16


def irx_tail() -> bool:
    """``ARENA_IRX_TAIL`` (default 0): with hidden slicing (``ARENA_IRX_SLICES`` > 1) the 14 -> 7 block and the
    7x7 blocks also run as the whole-map x3 kernel (one row band, hidden channels over workgroups, partial sums
    between blocks) instead of expand GEMM + depthwise + project GEMM."""
    if os.environ.get("ARENA_IRX_TAIL", "0").lower() in ("0", "false", "no", "off"):
        return False
    try:
        return int(os.environ.get("ARENA_IRX_SLICES", "6")) > 1
    except ValueError:
        return True


def ir_crop_f32_planned(H: int, stride: int, inp_pad: int, hid_pad: int, oup_pad: int, expand: int) -> bool:
    from .validate import ir_crop_f32_supported

    policy = ir_crop_f32_policy()
    if policy == "none" or (policy == "auto" and not (H == 14 and stride == 1) and not (irx_tail() and H in (14, 7))):
        return False
    return ir_crop_f32_supported(H, stride, inp_pad, hid_pad, oup_pad, expand)


class ProgramBuilder:
    _lane = 0

    def __init__(self, dtype: str = "bf16") -> None:
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")
        self.dtype = dtype
        self.f32 = dtype == "fp32"
        self.elem = 4 if self.f32 else 2
        self.buffers: list[Buffer] = []
        self.ops: list[list[int]] = []
        self.cls_start: int | None = None
        self.weights = WeightPacker()
        self.meta: dict = {"dtype": dtype}

    def _bf16_only(self, what: str) -> None:
        if self.f32:
            raise ValueError(f"{what} is a bf16-only fused kernel; fp32 programs use the unfused ops")

    # ------------------------------------------------------------ buffers
    def tensor(self, name: str, H: int, W: int, C: int, kind: int = IMAGES, elem: int | None = None) -> Buffer:
        elem = self.elem if elem is None else elem
        if C % 8:
            raise ValueError(f"{name}: channel count {C} must be a multiple of 8")
        b = Buffer(len(self.buffers), name, _round(H * W * C * elem, 16), kind, H, W, C, elem)
        self.buffers.append(b)
        return b

    def raw(self, name: str, per_item: int, kind: int = IMAGES, pinned: bool = False) -> Buffer:
        b = Buffer(len(self.buffers), name, _round(per_item, 16), kind, pinned=pinned)
        self.buffers.append(b)
        return b

    def _touch(self, *views) -> None:
        i = len(self.ops)
        for v in views:
            if v is None:
                continue
            b = v.buf if isinstance(v, View) else v
            if isinstance(b, Buffer):
                b.first = min(b.first, i)
                b.last = max(b.last, i)

    def _emit(self, rec: list[int], *touch) -> None:
        self._touch(*touch)
        if len(rec) > OP_LANE_FIELD:
            raise ValueError("op record overlaps the lane / dtype fields")
        r = list(rec) + [0] * (OP_FIELDS - len(rec))
        r[OP_DTYPE_FIELD] = int(self.f32)
        r[OP_LANE_FIELD] = self._lane
        self.ops.append(r)

    def parallel(self):
        """Context for a region of independent branches: ``with pb.parallel() as lane: lane(1); ...ops...;
        lane(2); ...``.  Each branch's ops carry its lane (OP_LANE_FIELD) and run on a side stream of the batch
        (executor.cpp enqueue_program: forked before the region, joined at the next lane-0 op).  Every buffer the
        region touches stays allocated for the whole region: the arena layout must not let two branches share
        memory they now use at the same time."""
        import contextlib

        @contextlib.contextmanager
        def region():
            start = len(self.ops)

            def lane(k: int) -> None:
                if not 0 <= k <= MAX_LANES:
                    raise ValueError(f"lane {k} outside 0..{MAX_LANES}")
                self._lane = k

            try:
                yield lane
            finally:
                self._lane = 0
                end = len(self.ops)
                if not any(self.ops[i][OP_LANE_FIELD] for i in range(start, end)):
                    return  # every branch on the main stream: sequential lifetimes stay valid
                for b in self.buffers:
                    if b.last >= start and b.first < end:
                        b.first = min(b.first, start)
                        b.last = max(b.last, end - 1)

        return region()

    def begin_classifier(self) -> None:
        """Ops from here on form the overflow classification program."""
        self.cls_start = len(self.ops)

    # ------------------------------------------------------------ ops
    def conv(self, src: View, dst: View, w: torch.Tensor, b: torch.Tensor, *, stride: int = 1,
             pad: int | tuple[int, int] | None = None, act: str | None = "silu", res: View | None = None,
             dst2: View | None = None, f32out: bool = False, kind: int = IMAGES,
             out_hw: tuple[int, int] | None = None, src_hw: tuple[int, int] | None = None,
             raw_cs: int | None = None, pw: tuple | None = None) -> None:
        """``pw=(w2, b2, dst2_view, act2)``: a 1x1 conv applied to this conv's activated output inside the
        kernel epilogue (the 3x3 result is not stored when ``dst`` is ``View(BUF_NONE, 0, Cout)``)."""
        cout, cin, kh, kw = w.shape
        if cin != src.C:
            raise ValueError(f"conv: weight Cin {cin} != source view C {src.C}")
        if cout != dst.C:
            raise ValueError(f"conv: weight Cout {cout} != destination view C {dst.C}")
        dst_cs = dst.cs if raw_cs is None else int(raw_cs)
        H, W = src_hw if src_hw else (src.buf.H, src.buf.W)
        if pad is None:
            pad = (kh // 2, kw // 2)
        if isinstance(pad, int):
            pad = (pad, pad)
        if out_hw is None:
            Ho = (H + 2 * pad[0] - kh) // stride + 1
            Wo = (W + 2 * pad[1] - kw) // stride + 1
        else:
            Ho, Wo = out_hw
        wb, bb, kpad, cpad = pack_conv_weight(w, b, self.dtype)
        w_off = self.weights.add(wb)
        b_off = self.weights.add(bb)
        rec = [OP_CONV, src.bid, src.coff, src.cs, H, W, cin, w_off, kpad, b_off,
               dst.bid, dst.coff, dst_cs, Ho, Wo, cout, cpad, kh, kw, stride, pad[0], pad[1],
               res.bid if res else BUF_NONE, res.coff if res else 0, res.cs if res else 0,
               dst2.bid if dst2 else BUF_NONE, dst2.coff if dst2 else 0, dst2.cs if dst2 else 0,
               ACT[act], int(f32out), kind]
        pw_dst = None
        if pw is not None:
            w2, b2, pw_dst, act2 = pw
            co2, ci2 = w2.shape[0], w2.shape[1]
            if ci2 != cout or w2.shape[2:] != (1, 1) or co2 != pw_dst.C:
                raise ValueError("conv: fused pointwise weights must be [C2, Cout, 1, 1] with C2 == pw dst C")
            if self.f32:  # x3hg epilogue: pre-split 1x1 planes, the 3x3 itself as x3g planes (fields 40-41)
                if (kh, kw, stride) != (3, 3, 1):
                    raise ValueError("conv: the fp32 fused pointwise epilogue needs a 3x3 stride-1 conv")
                kpad2, cpad2 = _round(cout, 32), _round(co2, 16)
                wb2 = pack_pw_weight_x3(w2, kpad2)
                bb2 = torch.zeros(cpad2)
                bb2[:co2] = b2.detach().float()
                bb2 = bb2.numpy().tobytes()
            else:
                wb2, bb2, kpad2, cpad2 = pack_conv_weight(w2, b2)
            rec += [self.weights.add(wb2), kpad2, self.weights.add(bb2), co2, cpad2, pw_dst.bid, pw_dst.coff,
                    pw_dst.cs, ACT[act2]]
            if self.f32:
                rec += [self.weights.add(pack_conv_weight_x3(w)), 1]
        elif self.f32 and src.bid != BUF_POOL:
            # fp32: the weights once more as pre-split bf16 planes for the x3g kernels (fields 40-41)
            rec += [0] * 9 + [self.weights.add(pack_conv_weight_x3(w)), 1]
        self._emit(rec, src, dst, res, dst2, pw_dst)

    def dwconv(self, src: View, dst: View, w: torch.Tensor, b: torch.Tensor, *, stride: int, act: str = "relu6",
               kind: int = IMAGES) -> None:
        C = w.shape[0]
        if w.shape[1:] != (1, 3, 3) or src.C != C or dst.C != C:
            raise ValueError("dwconv: expects [C,1,3,3] weights matching the views")
        H, W = src.buf.H, src.buf.W
        Ho, Wo = (H + 2 - 3) // stride + 1, (W + 2 - 3) // stride + 1
        wt = w.detach().float().reshape(C, 9).t().contiguous()  # [9][C]
        w_off = self.weights.add(f32_bytes(wt) if self.f32 else bf16_bytes(wt))
        b_off = self.weights.add(b.detach().float().numpy().tobytes())
        rec = [OP_DWCONV, src.bid, src.coff, src.cs, H, W, C, w_off, b_off, dst.bid, dst.coff, dst.cs,
               Ho, Wo, stride, ACT[act], kind]
        self._emit(rec, src, dst)

    def ir_block(self, src: View, dst: View, expand, dw, project, *, stride: int, res: bool,
                 kind: int = CROPS, x_parts: int = 1, y_parts: int = 1) -> None:
        """Fused inverted residual: ``expand`` = (w [hid,inp,1,1], b) or None (t = 1 blocks),
        ``dw`` = (w [hid,1,3,3], b), ``project`` = (w [oup,hid,1,1], b); BN already folded.

        ``x_parts`` / ``y_parts`` > 1 (fp32 14x14 whole-map blocks, csrc/kernels/ir_crop_f32.hip): the source view
        holds ``x_parts`` partial sums of the block input side by side (C = x_parts * inp), and the block's hidden
        channels are split over ``y_parts`` workgroups per row band that write ``y_parts`` partial outputs
        (dst C = y_parts * oup) — the next block adds them while loading its input."""
        if dst.C != project[0].shape[0] * y_parts:
            raise ValueError(f"ir_block: destination C {dst.C} != oup {project[0].shape[0]} x {y_parts} parts")
        pk = pack_ir_weights(expand, dw, project, src.C // max(1, x_parts), k_align=16 if self.f32 else 32)
        inp, inp_pad, hid_pad, oup, oup_pad = pk["inp"], pk["inp_pad"], pk["hid_pad"], pk["oup"], pk["oup_pad"]
        f32 = lambda t: t.float().contiguous().numpy().tobytes()  # noqa: E731
        mat = f32 if self.f32 else bf16_bytes  # exact-fp32 programs keep fp32 weights
        H, W = src.buf.H, src.buf.W
        # fp32 14x14 / 7x7 blocks: whole-map kernel with pre-split [h|m|l] bf16 expand / project weights
        x3w = 0
        if self.f32:
            x3w, inp_x3 = ir_x3_plan(H, W, stride, inp, hid_pad, oup_pad, int(expand is not None))
            if x3w and inp_x3 != inp_pad:  # the x3 kernels step K by 32
                pk = pack_ir_weights(expand, dw, project, src.C // max(1, x_parts), k_align=32)
                inp, inp_pad, hid_pad, oup, oup_pad = pk["inp"], pk["inp_pad"], pk["hid_pad"], pk["oup"], \
                    pk["oup_pad"]
        mat_x3 = (lambda t: bf16_raw_bytes(split_bf16x3(t))) if x3w else mat  # noqa: E731
        offs = [self.weights.add(mat_x3(pk["we"])), self.weights.add(f32(pk["be"])),
                self.weights.add(mat(pk["wd"])), self.weights.add(f32(pk["bd"])),
                self.weights.add(mat_x3(pk["wp"])), self.weights.add(f32(pk["bp"]))]
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        if (x_parts > 1 or y_parts > 1) and not (x3w and H == W and H in (14, 7) and inp % 4 == 0
                                                 and src.C == inp * x_parts and y_parts <= hid_pad // 32 and max(x_parts, y_parts) <= 8):
            raise ValueError("ir_block: partial-sum tensors need the fp32 14x14 whole-map kernel")
        rec = [OP_IRBLOCK, src.bid, src.coff, src.cs, H, W, inp, inp_pad, hid_pad, oup, oup_pad, stride,
               int(expand is not None), int(res), *offs, dst.bid, dst.coff, dst.cs, Ho, Wo, kind, x3w,
               int(x_parts) if x_parts > 1 else 0, int(y_parts) if y_parts > 1 else 0]
        self._emit(rec, src, dst)

    def ir_block_stem(self, crops: Buffer, dst: View, stem, dw, project, *, S: int, mean, std,
                      kind: int = CROPS) -> None:
        """fp32 classifier front end in one op: crop gather + ImageNet normalisation -> space-to-depth -> the
        2x2 stem conv (``stem`` = (w [32, 16, 2, 2] over the s2d input, b), ReLU6) -> MobileNetV2 block 1 (t = 1:
        ``dw`` depthwise 32 + ReLU6, ``project`` 32 -> 16); ``dst`` is the block output (S/2 x S/2 x 16).  Neither
        the s2d crops nor the 112 x 112 x 32 stem map is stored (csrc/kernels/ir_f32.hip, IrParams.stem)."""
        if not self.f32:
            raise ValueError("ir_block_stem is an fp32-program op (bf16 programs use stem_fused)")
        ws, bs = stem
        if ws.shape != (32, 16, 2, 2) or dw[0].shape != (32, 1, 3, 3) or project[0].shape[1:] != (32, 1, 1) \
                or project[0].shape[0] != dst.C or dst.C > 16 or S % 2:
            raise ValueError("ir_block_stem: needs a [32,16,2,2] s2d stem, a 32-channel t = 1 block and <= 16 outputs")
        pk = pack_ir_weights(None, dw, project, 32, k_align=16)
        f32 = lambda t: t.float().contiguous().numpy().tobytes()  # noqa: E731
        # x3w: stem and project weights as split bf16 planes for csrc/kernels/ir_tile_x3.hip (ARENA_STEM_X3)
        x3w = int(stem_x3_enabled())
        mat_x3 = (lambda t: bf16_raw_bytes(split_bf16x3(t.float()))) if x3w else f32  # noqa: E731
        offs = [self.weights.add(mat_x3(pk["we"])), self.weights.add(f32(pk["be"])), self.weights.add(f32(pk["wd"])),
                self.weights.add(f32(pk["bd"])), self.weights.add(mat_x3(pk["wp"])), self.weights.add(f32(pk["bp"]))]
        wsb, bsb, kpad, cpad = pack_conv_weight(ws, bs, "fp32")
        if kpad != 64 or cpad != 32:
            raise ValueError("ir_block_stem: stem weights must pack to [32][64]")
        if x3w:
            # csrc/kernels/ir_tile_x3.hip ir_stem_x3_kernel stages the crop's uint8 values k, not the normalised
            # (k / 255 - mean_c) / std_c: the weights take the 1 / (255 std_c) of their input channel (s2d channel
            # ci = 3 pq + c) and the mean becomes a constant per (tap, output channel), added for the taps whose
            # s2d pixel lies inside the map.  fp64 here, rounded once to fp32.
            w64 = torch.frombuffer(bytearray(wsb), dtype=torch.float32).reshape(32, 64).double()
            ci = torch.arange(64) % 16
            live = ci < 12
            inv = torch.tensor([1.0 / (255.0 * float(std[c % 3])) for c in range(12)] + [0.0] * 4, dtype=torch.float64)
            mstd = torch.tensor([float(mean[c % 3]) / float(std[c % 3]) for c in range(12)] + [0.0] * 4,
                                dtype=torch.float64)
            w_int = torch.where(live[None, :], w64 * inv[ci][None, :], torch.zeros_like(w64))
            consts = torch.stack([-(w64[:, 16 * t:16 * t + 16] * mstd[None, :]).sum(1) for t in range(4)])  # [4][32]
            bias = torch.frombuffer(bytearray(bsb), dtype=torch.float32)[:32].double()
            bsb = torch.cat([bias, consts.reshape(-1)]).float().contiguous().numpy().tobytes()
            wsb = mat_x3(w_int.float())
        H = S // 2
        rec = [OP_IRBLOCK, BUF_NONE, 0, 0, H, H, 32, pk["inp_pad"], pk["hid_pad"], pk["oup"], pk["oup_pad"], 1, 0, 0,
               *offs, dst.bid, dst.coff, dst.cs, H, H, kind, x3w, 0, 0, 0, 0,
               1, crops.id, S] + [fbits(m) for m in mean] + [fbits(1.0 / s) for s in std] + \
              [self.weights.add(wsb), self.weights.add(bsb)]
        self._emit(rec, dst, crops)

    def sppf(self, buf: Buffer, C: int, kind: int = IMAGES) -> None:
        self._emit([OP_SPPF, buf.id, 0, buf.C, buf.H, buf.W, C, kind], buf)

    def letterbox(self, out: Buffer, T: int) -> None:
        self._emit([OP_LETTERBOX, out.id, T], out)

    def letterbox_conv(self, dst: View, w: torch.Tensor, b: torch.Tensor, *, T: int, act: str = "silu") -> None:
        """fp32 stem conv (3x3 s1 over the 16-channel space-to-depth grid) whose input is the letterboxed
        batch images themselves (source buffer BUF_POOL): the kernel samples the uint8 images as the letterbox
        op would, so the T/2 x T/2 x 16 fp32 input tensor is never materialised (executor OP_CONV, x3-h16)."""
        if not self.f32:
            raise ValueError("letterbox_conv: fp32 programs only (bf16 programs use stem_fused)")
        if w.shape[1:] != (16, 3, 3) or T % 2:
            raise ValueError("letterbox_conv: expects [Cout, 16, 3, 3] weights and an even target size")
        self.conv(View(BUF_POOL, 0, 16), dst, w, b, act=act, src_hw=(T // 2, T // 2))

    def c3_fused(self, src: View, dst: View, H: int, W: int, cv12: tuple, bottlenecks: list, cv3: tuple, *,
                 res: bool, kind: int = IMAGES) -> None:
        """A whole C3 block as one op: ``cv12`` = (w, b) of cv1|cv2 stacked [2CH, C1, 1, 1]; ``bottlenecks`` =
        [((w1, b1), (w2, b2)), ...] with w1 [CH, CH, 1, 1], w2 [CH, CH, 3, 3]; ``cv3`` = (w, b) [2CH, 2CH, 1, 1].
        fp32 programs: the 160x160 block only (C1 32, CH 16, one bottleneck with shortcut), weights as pre-split
        bf16 planes for csrc/kernels/c3_x3.hip."""
        w12, b12 = cv12
        ch2, c1 = w12.shape[0], w12.shape[1]
        CH, NB = ch2 // 2, len(bottlenecks)
        if c1 != src.C or dst.C != ch2 or not 1 <= NB <= 2:
            raise ValueError("c3_fused: channel / bottleneck count mismatch")
        rec = [OP_C3FUSED, src.bid, src.coff, src.cs, H, W, c1, CH, NB, int(res)]
        if self.f32:
            if (c1, CH, NB, bool(res)) != (32, 16, 1, True) or H % 8 or W % 16:
                raise ValueError("c3_fused: the fp32 kernel takes the 160x160 block (C1 32, c_ 16, n 1, shortcut)")
            x3 = lambda t: bf16_raw_bytes(split_bf16x3(t))  # noqa: E731
            (w1, b1), (w2, b2) = bottlenecks[0]
            w2k = torch.zeros(CH, 160)  # k = (ky * 3 + kx) * CH + ci, 144 -> 160 (five 32-deep K steps)
            w2k[:, :9 * CH] = w2.detach().float().permute(0, 2, 3, 1).reshape(CH, 9 * CH)
            w3, b3 = cv3
            parts = [x3(w12.reshape(ch2, c1)), f32_bytes(b12)]
            parts += [x3(w1.reshape(CH, CH)), f32_bytes(b1), x3(w2k), f32_bytes(b2)] * 2  # slot 1 unused (NB 1)
            parts += [x3(w3.reshape(ch2, ch2)), f32_bytes(b3)]
            rec += [self.weights.add(b) for b in parts] + [dst.bid, dst.coff, dst.cs, kind]
            self._emit(rec, src, dst)
            return
        wb, bb, _, _ = pack_conv_weight(w12, b12)
        rec += [self.weights.add(wb), self.weights.add(bb)]
        for k in range(2):
            (w1, b1), (w2, b2) = bottlenecks[min(k, NB - 1)]
            w1p = torch.zeros(CH, 32, 1, 1)  # [CH][32]: k >= CH columns zero (the kernel reads T's first 32 ch)
            w1p[:, :CH] = w1.reshape(CH, CH, 1, 1)
            wa, ba, _, _ = pack_conv_weight(w1p, b1)
            wc, bc, _, _ = pack_conv_weight(w2, b2)
            rec += [self.weights.add(wa), self.weights.add(ba), self.weights.add(wc), self.weights.add(bc)]
        w3, b3 = cv3
        wd, bd, _, _ = pack_conv_weight(w3, b3)
        rec += [self.weights.add(wd), self.weights.add(bd), dst.bid, dst.coff, dst.cs, kind]
        self._emit(rec, src, dst)

    def stem_fused(self, dst: View, w: torch.Tensor, b: torch.Tensor, *, S: int, act: str, crops: Buffer | None = None,
                   mean=None, std=None, kind: int = IMAGES, second: tuple | None = None,
                   ir: tuple | None = None) -> None:
        """Letterbox (``crops=None``) or crop gather + normalisation, fused with the s2d stem conv
        (``w``: [Cout, 16, KS, KS] over the space-to-depth input, pad top/left 1).

        ``second=(w2, b2, act2)`` (detector only): the following 3x3 stride-2 conv runs in the same
        kernel on the stem output kept in LDS; ``dst`` is then that conv's output (S/4 x S/4).
        ``ir=(dw, project)`` (classifier only): MobileNetV2 block 1 (t = 1, 32 -> 16, stride 1, no
        residual) runs on the stem output in LDS; ``dst`` is then the block's output (S/2 x S/2 x 16)."""
        if self.f32 and (second is None or crops is not None or ir is not None):
            raise ValueError("stem_fused: the fp32 form is letterbox + stem + 3x3 s2 conv (csrc/kernels/stem_x3.hip)")
        cout, cin, ks, ks2 = w.shape
        if cin != 16 or ks != ks2:
            raise ValueError("stem_fused: weights must be [Cout, 16, KS, KS]")
        wb, bb, kpad, cpad = pack_conv_weight(w, b)
        if cpad != cout:
            raise ValueError("stem_fused: Cout must be a multiple of 16")
        if self.f32:
            if (cout, ks, second[0].shape) != (16, 3, (32, 16, 3, 3)):
                raise ValueError("stem_fused: the fp32 kernel takes a 3x3 16 -> 16 stem and a 3x3 s2 16 -> 32 conv")
            wb, wb2_x3 = pack_stem_s2_x3(w, second[0])
        w_off = self.weights.add(wb)
        b_off = self.weights.add(bb)
        src = 0 if crops is None else 1
        mean = mean if mean is not None else (0.0, 0.0, 0.0)
        std = std if std is not None else (1.0, 1.0, 1.0)
        if second is not None:
            w2, b2, act2 = second
            co2, ci2, kh2, kw2 = w2.shape
            if crops is not None or ci2 != cout or (kh2, kw2) != (3, 3) or co2 != dst.C:
                raise ValueError("stem_fused: second conv must be 3x3 [C2, Cout, 3, 3] with C2 == dst.C")
        elif ir is not None:
            (wd, _), (wp, _) = ir
            if crops is None or wd.shape != (cout, 1, 3, 3) or wp.shape[1:] != (cout, 1, 1) or wp.shape[0] != dst.C \
                    or cout != 32 or dst.C != 16:
                raise ValueError("stem_fused: fused block must be depthwise [32,1,3,3] + project [16,32,1,1]")
        elif cout != dst.C:
            raise ValueError("stem_fused: Cout must match dst.C")
        rec = [OP_STEMFUSED, src, dst.bid, dst.coff, dst.cs, S, w_off, kpad, b_off, cout, ACT[act],
               crops.id if crops is not None else BUF_NONE] + [fbits(m) for m in mean] + \
              [fbits(1.0 / s) for s in std] + [kind, ks]
        if second is not None:
            wb2, bb2, kpad2, _ = pack_conv_weight(w2, b2)
            if self.f32:
                wb2 = wb2_x3
            rec += [1, self.weights.add(wb2), kpad2, self.weights.add(bb2), co2, ACT[act2]]
        else:
            rec += [0] * 6
        if ir is not None:
            pk = pack_ir_weights(None, ir[0], ir[1], cout)
            f32 = lambda t: t.float().contiguous().numpy().tobytes()  # noqa: E731
            rec += [1, self.weights.add(bf16_bytes(pk["wd"])), self.weights.add(f32(pk["bd"])),
                    self.weights.add(bf16_bytes(pk["wp"])), self.weights.add(f32(pk["bp"])), pk["oup"]]
        self._emit(rec, dst, crops)

    def stamp(self, k: int) -> None:
        if not 0 <= k < 4:
            raise ValueError("stamp index must be 0..3")
        self._emit([OP_STAMP, int(k)])

    def zero(self, buf: Buffer, kind: int = IMAGES) -> None:
        self._emit([OP_ZERO, buf.id, buf.per_item, kind], buf)

    def decode(self, heads: list[View], strides, cand: Buffer, count: Buffer, conf_thr: float) -> None:
        rec = [OP_DECODE]
        for v in heads:
            rec += [v.bid, v.coff, v.cs, v.buf.H]
        rec += list(int(s) for s in strides) + [cand.id, count.id, fbits(conf_thr)]
        self._emit(rec, *heads, cand, count)

    def nms(self, cand: Buffer, count: Buffer, iou_thr: float) -> None:
        self._emit([OP_NMS, cand.id, count.id, BUF_DET, BUF_DETCOUNT, fbits(iou_thr)], cand, count)

    def crop_plan(self, crops: Buffer, whole: bool = False) -> None:
        self._emit([OP_CROPPLAN, BUF_DET, BUF_DETCOUNT, crops.id, int(whole)], crops)

    def tensor_in(self, out: Buffer, S: int) -> None:
        self._emit([OP_TENSORIN, out.id, S], out)

    def yolo_raw(self, heads: list[View], strides) -> None:
        rec = [OP_YOLORAW]
        for v in heads:
            rec += [v.bid, v.coff, v.cs, v.buf.H]
        rec += list(int(s) for s in strides) + [BUF_RAWOUT]
        self._emit(rec, *heads)

    def crop_gather(self, crops: Buffer, out: Buffer, S: int, mean, std) -> None:
        rec = [OP_CROPGATHER, crops.id, out.id, S] + [fbits(m) for m in mean] + [fbits(1.0 / s) for s in std]
        self._emit(rec, crops, out)

    def head_pool(self, src: View, dst: View, w: torch.Tensor, b: torch.Tensor, *, act: str | None = "relu6",
                  kind: int = CROPS) -> None:
        """1x1 conv + activation + global average pool in one kernel: ``dst`` is a 1x1 map (bf16:
        csrc/kernels/head_pool.hip head_pool; fp32: head_pool_f32, triple-bf16-split MFMA)."""
        cout, cin, kh, kw = w.shape
        if (kh, kw) != (1, 1) or cin != src.C or cout != dst.C or dst.buf.H * dst.buf.W != 1:
            raise ValueError("head_pool: expects 1x1 weights [N, C, 1, 1] and a 1x1 destination")
        wb, bb, kpad, cpad = pack_conv_weight(w, b, self.dtype)
        rec = [OP_HEADPOOL, src.bid, src.coff, src.cs, src.buf.H * src.buf.W, cin, self.weights.add(wb), kpad,
               self.weights.add(bb), cout, cpad, dst.bid, dst.coff, dst.cs, ACT[act], kind]
        self._emit(rec, src, dst)

    def avgpool(self, x: Buffer, y: Buffer, kind: int = CROPS) -> None:  # noqa: D401
        self._emit([OP_AVGPOOL, x.id, x.H * x.W, x.C, y.id, kind], x, y)

    def topk(self, logits: Buffer, N: int, ld: int) -> None:
        self._emit([OP_TOPK, logits.id, N, ld, BUF_TOPK], logits)

    # ------------------------------------------------------------ finalize
    def build(self, meta: dict | None = None) -> Program:
        n = len(self.ops)
        for b in self.buffers:
            if b.pinned and b.last >= 0:
                b.last = n
        ops = np.asarray(self.ops, dtype=np.int64).reshape(n, OP_FIELDS)
        cs = self.cls_start if self.cls_start is not None else n
        cls_ops = ops[cs:].copy()
        m = dict(self.meta)
        m.update(meta or {})
        return Program(ops, cls_ops, self.buffers, self.weights.blob(), m)


def layout(buffers: list[Buffer], n_images: int, n_crops: int, share: bool = True) -> tuple[np.ndarray, int]:
    """Lifetime-aware first-fit placement; returns (offsets per buffer id, arena bytes).

    ``share=False`` gives every buffer its own range (debugging: every
    intermediate tensor stays readable after a run).
    """
    sizes = []
    for b in buffers:
        cnt = n_crops if b.kind == CROPS else n_images
        sizes.append(_round(b.per_item * cnt, ALIGN))
    order = sorted(range(len(buffers)), key=lambda i: (-sizes[i], buffers[i].first))
    placed: list[tuple[int, int, int]] = []  # (offset, end, id)
    offsets = np.zeros(len(buffers), dtype=np.int64)
    total = 0
    for i in order:
        b = buffers[i]
        if b.last < 0:  # never used
            offsets[i] = 0
            continue
        conflicts = sorted(
            (o, e) for (o, e, j) in placed
            if not share or not (buffers[j].last < b.first or b.last < buffers[j].first)
        )
        off = 0
        for o, e in conflicts:
            if off + sizes[i] <= o:
                break
            off = max(off, e)
        offsets[i] = off
        placed.append((off, off + sizes[i], i))
        total = max(total, off + sizes[i])
    return offsets, _round(total, ALIGN)
