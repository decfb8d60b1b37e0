"""Static bounds check of an executor program (runs on the CPU).

Before a program is captured into a hipGraph, every op's device accesses are
replayed symbolically against the buffer sizes of a bucket layout: each
(view, pixel count, channel slice) must stay inside its buffer.  This catches
planner bugs as exceptions on the host instead of GPU faults.
"""
from __future__ import annotations

from ..engine.planner import (
    BUF_CTRL,
    BUF_DET,
    BUF_DETCOUNT,
    BUF_META,
    BUF_NONE,
    BUF_POOL,
    BUF_RAWOUT,
    BUF_TOPK,
    BUF_XCROPS,
    CROPS,
    OP_AVGPOOL,
    OP_C3FUSED,
    OP_HEADPOOL,
    OP_CONV,
    OP_CROPGATHER,
    OP_CROPPLAN,
    OP_DECODE,
    OP_DWCONV,
    OP_IRBLOCK,
    OP_LETTERBOX,
    OP_NMS,
    OP_SPPF,
    OP_STAMP,
    OP_STEMFUSED,
    OP_TENSORIN,
    OP_TOPK,
    OP_YOLORAW,
    OP_ZERO,
    OP_DTYPE_FIELD,
    Program,
)

CAND_BYTES, DET_BYTES, CROP_BYTES, TOPK_BYTES = 32, 32, 32, 64


class ProgramError(ValueError):
    pass


def ir_f32_lds_bytes(stride: int, inp_pad: int, expand: bool) -> int:
    """LDS of one csrc/kernels/ir_f32.hip workgroup (must mirror irf_lds_bytes)."""
    th, tw = (8, 8) if stride == 1 else (4, 8)
    ph, pw = (th - 1) * stride + 3, (tw - 1) * stride + 3
    rows = (ph * pw + 15) // 16 * 16
    xp = inp_pad + 8 if expand else inp_pad
    ep = 32 if stride == 1 else 36
    return 4 * (rows * xp + (rows * ep if expand else 0) + th * tw * 40 + rows)


def ir_f32_supported(stride: int, inp_pad: int, hid_pad: int, oup_pad: int, expand: int) -> bool:
    """Mirror of arena::ir_block_f32_supported."""
    return (stride in (1, 2) and inp_pad % 16 == 0 and inp_pad <= 64 and hid_pad % 32 == 0 and oup_pad % 16 == 0
            and oup_pad // 16 in (1, 2, 4, 6) and (bool(expand) or hid_pad == inp_pad)
            and ir_f32_lds_bytes(stride, inp_pad, bool(expand)) <= 64 * 1024)


# (output side, stride, inp_pad, oup_pad) of csrc/kernels/ir_crop_f32.hip ARENA_IRX_CONFIGS (hidden chunks of 32)
IR_CROP_F32_CONFIGS = {(14, 1, 64, 64), (14, 1, 64, 96), (14, 1, 96, 96), (7, 2, 96, 160), (7, 1, 160, 160),
                       (7, 1, 160, 320)}


# (stride, oup_pad, inp_pad) of csrc/kernels/ir_tile_x3.hip ITX_CONFIGS
IR_TILE_X3_CONFIGS = {(1, 16, 32), (1, 32, 32), (1, 64, 32), (1, 32, 64), (1, 64, 64), (2, 16, 32), (2, 32, 32),
                      (2, 64, 32), (2, 64, 64)}


def ir_tile_x3_supported(stride: int, inp_pad: int, hid_pad: int, oup_pad: int, expand: int) -> bool:
    """Mirror of arena::ir_tile_x3_supported (tiled x3 block kernel for the >= 28x28 stages)."""
    return bool(expand) and hid_pad % 32 == 0 and (stride, oup_pad, inp_pad) in IR_TILE_X3_CONFIGS


def ir_crop_f32_supported(H: int, stride: int, inp_pad: int, hid_pad: int, oup_pad: int, expand: int) -> bool:
    """Mirror of arena::ir_block_crop_f32_supported (whole-map x3 kernel for the 14x14 / 7x7 stages)."""
    Ho = (H - 1) // stride + 1
    return (bool(expand) and hid_pad % 32 == 0 and H == Ho * stride
            and (Ho, stride, inp_pad, oup_pad) in IR_CROP_F32_CONFIGS)


def validate_program(prog: Program, B: int, crop_cap: int, *, max_det: int, cand_cap: int,
                     raw_out_bytes: int | None = None) -> None:
    sizes = {}
    for b in prog.buffers:
        sizes[b.id] = b.per_item * (crop_cap if b.kind == CROPS else B)
    sizes[BUF_DET] = B * max_det * DET_BYTES
    sizes[BUF_DETCOUNT] = B * 4
    sizes[BUF_TOPK] = B * max_det * TOPK_BYTES
    sizes[BUF_XCROPS] = B * max_det * CROP_BYTES
    raw = int(raw_out_bytes if raw_out_bytes is not None else prog.meta.get("raw_out_bytes", 0))
    sizes[BUF_RAWOUT] = B * raw
    wbytes = prog.weights.nbytes
    names = {b.id: b.name for b in prog.buffers}

    def need(i, buf, lo, hi, what):
        if buf in (BUF_CTRL, BUF_META, BUF_POOL):
            return
        if buf == BUF_NONE:
            raise ProgramError(f"op {i}: {what} has no buffer")
        cap = sizes.get(buf)
        if cap is None:
            raise ProgramError(f"op {i}: {what} references unknown buffer {buf}")
        if lo < 0 or hi > cap:
            raise ProgramError(f"op {i}: {what} accesses bytes [{lo}, {hi}) of {names.get(buf, buf)} ({cap} bytes)")

    def view(i, buf, coff, cs, npix, C, elem, what):
        if buf == BUF_NONE:
            return
        if cs < coff + C:
            raise ProgramError(f"op {i}: {what} slice [{coff}, {coff + C}) exceeds pixel stride {cs}")
        need(i, buf, coff * elem, ((npix - 1) * cs + coff + C) * elem, what)

    def weights(i, off, n, what):
        if off < 0 or off + n > wbytes:
            raise ProgramError(f"op {i}: {what} reads weights [{off}, {off + n}) of {wbytes}")

    fused = ()  # bf16-only fused kernels (fp32 stem_fused: the letterbox + stem + s2 conv form only; fp32 C3: 160x160)
    for i, r in enumerate(prog.ops):
        op = int(r[0])
        kind_n = lambda k: crop_cap if int(k) == CROPS else B  # noqa: E731
        f32 = int(r[OP_DTYPE_FIELD]) == 1
        if int(r[OP_DTYPE_FIELD]) not in (0, 1):
            raise ProgramError(f"op {i}: bad dtype field {int(r[OP_DTYPE_FIELD])}")
        if f32 and op in fused:
            raise ProgramError(f"op {i}: fused op {op} has no fp32 kernel")
        el = 4 if f32 else 2  # activation bytes
        if op == OP_CONV:
            n = kind_n(r[30])
            H, W, Cin, Ho, Wo, Cout, Cpad, KH, KW = (int(v) for v in (r[4], r[5], r[6], r[13], r[14], r[15], r[16],
                                                                      r[17], r[18]))
            kpad = int(r[8])
            if kpad < KH * KW * Cin or kpad % (16 if f32 else 32) or Cpad % 16 or Cout > Cpad:
                raise ProgramError(f"op {i}: bad conv geometry")
            if f32 and (Cin < 16 or Cin % 4 or (int(r[34]) > 0 and int(r[41]) != 1)):
                raise ProgramError(f"op {i}: unsupported fp32 conv geometry")
            if int(r[1]) == BUF_POOL:  # letterbox-source stem (x3-h16 kernel samples the images)
                if not f32 or int(r[30]) == CROPS or (KH, KW, Cin, kpad, int(r[19]), int(r[20]), int(r[21])) != \
                        (3, 3, 16, 144, 1, 1, 1) or H != W or (Ho, Wo) != (H, W):
                    raise ProgramError(f"op {i}: letterbox-source conv must be an fp32 3x3 s1 conv over 16 channels")
            else:
                view(i, r[1], int(r[2]), int(r[3]), n * H * W, Cin, el, "conv input")
            oel = 4 if int(r[29]) else el
            view(i, r[10], int(r[11]), int(r[12]), n * Ho * Wo, Cout, oel, "conv output")
            view(i, r[22], int(r[23]), int(r[24]), n * Ho * Wo, Cout, el, "conv residual")
            view(i, r[25], int(r[26]), int(r[27]), n * 4 * Ho * Wo, Cout, el, "conv upsampled output")
            weights(i, int(r[7]), Cpad * kpad * el, "conv weight")
            weights(i, int(r[9]), Cpad * 4, "conv bias")
            if int(r[34]) > 0:  # fused pointwise epilogue
                co2, kpad2, cpad2 = int(r[34]), int(r[32]), int(r[35])
                if KH != 3 or KW != 3 or int(r[19]) != 1 or Cout not in (64, 80) or kpad2 != (Cout + 31) // 32 * 32 \
                        or co2 > Cout or int(r[22]) != BUF_NONE or int(r[25]) != BUF_NONE:
                    raise ProgramError(f"op {i}: unsupported fused pointwise geometry")
                view(i, r[36], int(r[37]), int(r[38]), n * Ho * Wo, co2, el, "fused pointwise output")
                # fp32: pre-split planes [round32(co2)][3][kpad2] (pack_pw_weight_x3); bf16: [cpad2][kpad2]
                wn = (co2 + 31) // 32 * 32 * 3 * kpad2 * 2 if f32 else cpad2 * kpad2 * 2
                weights(i, int(r[31]), wn, "pointwise weight")
                weights(i, int(r[33]), cpad2 * 4, "pointwise bias")
            if int(r[41]):  # pre-split bf16 weight planes (x3g / x3h kernels): [KH*KW*Cin32/32][Cout_pad][3][32]
                if not f32 or int(r[41]) != 1:
                    raise ProgramError(f"op {i}: pre-split weights belong to fp32 convs")
                weights(i, int(r[40]), KH * KW * ((Cin + 31) // 32) * Cpad * 192, "conv x3 weight")
        elif op == OP_DWCONV:
            n = kind_n(r[16])
            H, W, C, Ho, Wo = (int(v) for v in (r[4], r[5], r[6], r[12], r[13]))
            view(i, r[1], int(r[2]), int(r[3]), n * H * W, C, el, "dw input")
            view(i, r[9], int(r[10]), int(r[11]), n * Ho * Wo, C, el, "dw output")
            weights(i, int(r[7]), 9 * C * el, "dw weight")
            weights(i, int(r[8]), C * 4, "dw bias")
        elif op == OP_IRBLOCK:
            n = kind_n(r[25])
            H, W, inp, inp_pad, hid_pad, oup, oup_pad, S = (int(v) for v in r[4:12])
            Ho, Wo = int(r[23]), int(r[24])
            if inp_pad % (16 if f32 else 32) or hid_pad % 32 or oup_pad % 16 or inp > inp_pad or oup > oup_pad \
                    or inp % (4 if f32 else 8):
                raise ProgramError(f"op {i}: bad ir_block channel geometry")
            x3w = int(r[26])
            if any(int(v) for v in r[29:31]):
                raise ProgramError(f"op {i}: ir_block fields 29-30 are reserved (0)")
            xp, yp = max(1, int(r[27])), max(1, int(r[28]))
            if (xp > 1 or yp > 1) and not (f32 and x3w and H == W and H in (14, 7) and max(xp, yp) <= 8
                                           and yp <= hid_pad // 32 and inp % 4 == 0 and oup % 4 == 0):
                raise ProgramError(f"op {i}: partial-sum ir_block tensors need the fp32 14x14 whole-map kernel")
            if x3w and not (f32 and (int(r[31]) or (H == W and ir_crop_f32_supported(H, S, inp_pad, hid_pad, oup_pad,
                                                                                      int(r[12])))
                                     or ir_tile_x3_supported(S, inp_pad, hid_pad, oup_pad, int(r[12])))):
                raise ProgramError(f"op {i}: split-plane weights for a block no x3 kernel takes")
            if f32 and not x3w and not ir_f32_supported(S, inp_pad, hid_pad, oup_pad, int(r[12])):
                raise ProgramError(f"op {i}: no fp32 fused kernel for this block")
            if Ho != (H - 1) // S + 1 or Wo != (W - 1) // S + 1:
                raise ProgramError(f"op {i}: ir_block output size mismatch")
            if int(r[13]) and (S != 1 or inp != oup):
                raise ProgramError(f"op {i}: ir_block residual needs stride 1 and inp == oup")
            if int(r[31]):  # fp32 crop gather + stem computed in the kernel: no input view, the crop plan instead
                if not (f32 and S == 1 and not int(r[12]) and not int(r[13]) and inp == 32 and inp_pad == 32
                        and hid_pad == 32 and oup_pad == 16 and H == W and 2 * H == int(r[33]) and int(r[25]) == CROPS):
                    raise ProgramError(f"op {i}: unsupported fused stem + block geometry")
                need(i, r[32], 0, B * max_det * CROP_BYTES, "stem crop refs")
                weights(i, int(r[40]), 32 * 64 * (6 if x3w else 4), "stem weight")
                weights(i, int(r[41]), 32 * 4, "stem bias")
            else:
                view(i, r[1], int(r[2]), int(r[3]), n * H * W, inp * xp, el, "ir input")
            view(i, r[20], int(r[21]), int(r[22]), n * Ho * Wo, oup * yp, el, "ir output")
            wel = 6 if x3w else el  # three bf16 planes per weight
            weights(i, int(r[14]), hid_pad * inp_pad * wel, "ir expand weight")
            weights(i, int(r[15]), hid_pad * 4, "ir expand bias")
            weights(i, int(r[16]), 9 * hid_pad * el, "ir dw weight")
            weights(i, int(r[17]), hid_pad * 4, "ir dw bias")
            weights(i, int(r[18]), oup_pad * hid_pad * wel, "ir project weight")
            weights(i, int(r[19]), oup_pad * 4, "ir project bias")
        elif op == OP_SPPF:
            n = kind_n(r[7])
            if f32 and int(r[4]) * int(r[5]) > 512:
                raise ProgramError(f"op {i}: fp32 SPPF supports H*W <= 512")
            view(i, r[1], int(r[2]), int(r[3]), n * int(r[4]) * int(r[5]), 4 * int(r[6]), el, "sppf buffer")
        elif op == OP_LETTERBOX:
            T2 = int(r[2]) // 2
            need(i, r[1], 0, B * T2 * T2 * 16 * el, "letterbox output")
        elif op == OP_C3FUSED:
            n = kind_n(r[25])
            H, W, C1, CH, NB, res = (int(v) for v in r[4:10])
            ok = {(32, 16, 1, True)} if f32 else {(32, 16, 1, True), (64, 32, 2, True), (128, 32, 1, False)}
            if (C1, CH, NB, bool(res)) not in ok or H % 8 or W % 16:
                raise ProgramError(f"op {i}: unsupported fused C3 geometry {(C1, CH, NB, res, H, W)}")
            view(i, r[1], int(r[2]), int(r[3]), n * H * W, C1, el, "c3 input")
            view(i, r[22], int(r[23]), int(r[24]), n * H * W, 2 * CH, el, "c3 output")
            if f32:  # pre-split planes (c3_x3.hip): [2CH][3][C1], [CH][3][CH], [CH][3][160], [2CH][3][2CH]
                weights(i, int(r[10]), 2 * CH * 3 * C1 * 2, "c3 cv1|cv2 weight")
                weights(i, int(r[11]), 2 * CH * 4, "c3 cv1|cv2 bias")
                weights(i, int(r[12]), CH * 3 * CH * 2, "c3 bottleneck cv1 weight")
                weights(i, int(r[13]), CH * 4, "c3 bottleneck cv1 bias")
                weights(i, int(r[14]), CH * 3 * 160 * 2, "c3 bottleneck cv2 weight")
                weights(i, int(r[15]), CH * 4, "c3 bottleneck cv2 bias")
                weights(i, int(r[20]), 2 * CH * 3 * 2 * CH * 2, "c3 cv3 weight")
                weights(i, int(r[21]), 2 * CH * 4, "c3 cv3 bias")
                continue
            weights(i, int(r[10]), 2 * CH * C1 * 2, "c3 cv1|cv2 weight")
            weights(i, int(r[11]), 2 * CH * 4, "c3 cv1|cv2 bias")
            k3 = (9 * CH + 31) // 32 * 32
            for k in range(NB):
                weights(i, int(r[12 + 4 * k]), CH * 32 * 2, f"c3 bottleneck {k} cv1 weight")
                weights(i, int(r[13 + 4 * k]), CH * 4, f"c3 bottleneck {k} cv1 bias")
                weights(i, int(r[14 + 4 * k]), CH * k3 * 2, f"c3 bottleneck {k} cv2 weight")
                weights(i, int(r[15 + 4 * k]), CH * 4, f"c3 bottleneck {k} cv2 bias")
            weights(i, int(r[20]), 4 * CH * CH * 2, "c3 cv3 weight")
            weights(i, int(r[21]), 2 * CH * 4, "c3 cv3 bias")
        elif op == OP_STEMFUSED:
            src, S, kpad, cout, kind, ks = int(r[1]), int(r[5]), int(r[7]), int(r[9]), int(r[18]), int(r[19])
            n = kind_n(kind)
            expect = {0: (3, 16, 160, 0), 1: (2, 32, 64, CROPS)}.get(src)
            if expect is None or (ks, cout, kpad, kind) != expect or S % 2:
                raise ProgramError(f"op {i}: bad stem_fused geometry (src {src}, KS {ks}, Cout {cout}, Kpad {kpad})")
            if f32 and not int(r[20]):
                raise ProgramError(f"op {i}: an fp32 stem_fused op must carry the fused second conv")
            if int(r[20]):  # second conv fused: 3x3 s2 16 -> 32, output S/4
                if src != 0 or int(r[24]) != 32 or int(r[22]) != 160 or S % 64:
                    raise ProgramError(f"op {i}: bad fused second conv (Cout2 {int(r[24])}, Kpad2 {int(r[22])})")
                view(i, r[2], int(r[3]), int(r[4]), n * (S // 4) ** 2, 32, el, "stem second-conv output")
                # fp32 (stem_x3.hip): pre-split planes [9 taps][32][3][16]; bf16: [32][160]
                weights(i, int(r[21]), 9 * 32 * 3 * 16 * 2 if f32 else 32 * 160 * 2, "stem second-conv weight")
                weights(i, int(r[23]), 32 * 4, "stem second-conv bias")
            elif int(r[26]):  # first inverted residual fused: 32 -> 16 at S/2
                if src != 1 or int(r[31]) != 16 or S % 32:
                    raise ProgramError(f"op {i}: bad fused first block (oup {int(r[31])}, S {S})")
                view(i, r[2], int(r[3]), int(r[4]), n * (S // 2) ** 2, 16, 2, "stem first-block output")
                for off, nb, what in ((r[27], 9 * 32 * 2, "dw weight"), (r[28], 32 * 4, "dw bias"),
                                      (r[29], 16 * 32 * 2, "project weight"), (r[30], 16 * 4, "project bias")):
                    weights(i, int(off), nb, f"stem first-block {what}")
            else:
                view(i, r[2], int(r[3]), int(r[4]), n * (S // 2) ** 2, cout, 2, "stem output")
            if src == 1:
                need(i, r[11], 0, B * max_det * CROP_BYTES, "crop refs")
            # fp32: pre-split planes / 255 [3 ky][2 slabs][16][3][32]; bf16: [Cout][Kpad]
            weights(i, int(r[6]), 3 * 2 * 16 * 3 * 32 * 2 if f32 else cout * kpad * 2, "stem weight")
            weights(i, int(r[8]), cout * 4, "stem bias")
        elif op == OP_ZERO:
            need(i, r[1], 0, int(r[2]) * kind_n(r[3]), "zero")
        elif op == OP_DECODE:
            for lvl in range(3):
                buf, coff, cs, hw = (int(v) for v in r[1 + 4 * lvl: 5 + 4 * lvl])
                view(i, buf, coff, cs, B * hw * hw, 144, el, f"decode head {lvl}")
            need(i, r[16], 0, B * cand_cap * CAND_BYTES, "candidates")
            need(i, r[17], 0, B * 4, "candidate counts")
        elif op == OP_NMS:
            need(i, r[1], 0, B * cand_cap * CAND_BYTES, "nms candidates")
            need(i, r[3], 0, B * max_det * DET_BYTES, "nms detections")
        elif op == OP_CROPPLAN:
            need(i, r[3], 0, B * max_det * CROP_BYTES, "crop refs")
        elif op == OP_CROPGATHER:
            S2 = int(r[3]) // 2
            need(i, r[1], 0, B * max_det * CROP_BYTES, "crop refs")
            need(i, r[2], 0, crop_cap * S2 * S2 * 16 * el, "crop gather output")
        elif op == OP_HEADPOOL:
            n = kind_n(r[15])
            HW, K, Kpad, N, Npad = int(r[4]), int(r[5]), int(r[7]), int(r[9]), int(r[10])
            if not (0 < HW <= 64) or Kpad != 320 or K > Kpad or N % 4 or Npad % 16 or Npad < N:
                raise ProgramError(f"op {i}: head_pool geometry HW={HW} K={K} Kpad={Kpad} N={N} unsupported")
            view(i, r[1], int(r[2]), int(r[3]), n * HW, K, el, "head_pool input")
            weights(i, int(r[6]), Npad * Kpad * el, "head_pool weight")
            weights(i, int(r[8]), Npad * 4, "head_pool bias")
            view(i, r[11], int(r[12]), int(r[13]), n, N, el, "head_pool output")
        elif op == OP_AVGPOOL:
            n = kind_n(r[5])
            need(i, r[1], 0, n * int(r[2]) * int(r[3]) * el, "avgpool input")
            need(i, r[4], 0, n * int(r[3]) * el, "avgpool output")
        elif op == OP_TOPK:
            need(i, r[1], 0, crop_cap * int(r[3]) * 4, "topk logits")
            need(i, r[4], 0, B * max_det * TOPK_BYTES, "topk results")
        elif op == OP_TENSORIN:
            S2 = int(r[2]) // 2
            need(i, r[1], 0, B * S2 * S2 * 16 * el, "tensor input output")
        elif op == OP_YOLORAW:
            A = 0
            for lvl in range(3):
                buf, coff, cs, hw = (int(v) for v in r[1 + 4 * lvl: 5 + 4 * lvl])
                view(i, buf, coff, cs, B * hw * hw, 144, el, f"raw head {lvl}")
                A += hw * hw
            if int(r[16]) != BUF_RAWOUT or 84 * A * 4 > raw:
                raise ProgramError(f"op {i}: raw output needs {84 * A * 4} bytes per image, have {raw}")
        elif op == OP_STAMP:
            if not 0 <= int(r[1]) < 4:
                raise ProgramError(f"op {i}: stamp index {int(r[1])} out of range")
        else:
            raise ProgramError(f"op {i}: unknown op {op}")
