"""Tensor-level wrappers around the HIP kernels (torch tensors on ROCm).

These call the same launchers the executor uses, on the current torch stream,
so every kernel can be tested against a PyTorch fp32 reference op and used
outside the executor.  Activations are NHWC tensors — bf16 for the tuned bf16
kernels, float32 for the exact-fp32 kernels (selected by the input dtype); a
"view" into a concat buffer is passed as the buffer plus a channel offset.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np
import torch

from ..engine.planner import ACT, pack_conv_weight, pack_conv_weight_x3
from . import native

IMAGE_META = struct.Struct("<qiiiiiif12x")  # must match arena::ImageMeta (48 bytes)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None, elem_off: int = 0) -> int:
    if t is None:
        return 0
    return t.data_ptr() + elem_off * t.element_size()


def pack_weights(w: torch.Tensor, b: torch.Tensor, device, dtype: str = "bf16"):
    """-> (weights, bias, Kpad, Cout_pad, w3): ``w3`` the pre-split bf16 planes of the fp32 x3g kernels
    (planner.pack_conv_weight_x3; None for bf16)."""
    wb, bb, kpad, cpad = pack_conv_weight(w.detach().cpu().float(), b.detach().cpu().float(), dtype)
    wt = torch.frombuffer(bytearray(wb), dtype=torch.float32 if dtype == "fp32" else torch.bfloat16).to(device)
    bt = torch.frombuffer(bytearray(bb), dtype=torch.float32).to(device)
    w3 = None
    if dtype == "fp32":
        w3 = torch.frombuffer(bytearray(pack_conv_weight_x3(w.detach().cpu().float())), dtype=torch.int16).to(device)
    return wt, bt, kpad, cpad, w3


def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, *, stride: int = 1, pad=None, act=None,
                x_coff: int = 0, cin: int | None = None, out: torch.Tensor | None = None, out_coff: int = 0,
                res: torch.Tensor | None = None, res_coff: int = 0, out2: torch.Tensor | None = None,
                out2_coff: int = 0, f32out: bool = False, out_hw=None, bdev: torch.Tensor | None = None,
                packed=None, impl: int = 0, pw=None) -> torch.Tensor:
    """NHWC conv with fused bias/act/residual/upsampled copy.

    ``pw=(w2, b2)`` (fp32 3x3 stride-1 only): the Detect-head 1x1 ``w2`` [C2, Cout, 1, 1] is applied to the
    activated result inside the x3hg epilogue (impl 145 + v) and only its [B, Ho, Wo, C2] output is returned.

    x: [B, H, W, Cx] bf16 or float32 (reads channels [x_coff, x_coff + Cin)); w: [Cout, Cin, KH, KW] fp32.
    A float32 ``x`` runs the exact-fp32 kernel (fp32 weights, v_mfma_f32_16x16x4_f32, fp32 output).
    ``impl`` pins a kernel (0 = the dispatch policy; fp32: 1 direct, 2 LDS, 10 + v LDS tile variant v,
    40 + v triple-bf16-split variant v, 100 halo, 101 split halo, 102 / 103 split halo with 48 / 32-channel
    tiles, 104 / 105 weight-stationary streaming 1x1 (auto / 32-channel tiles), 111 + v the x3g 32x32x16 GEMM
    over pre-split weights — csrc/kernels/launch.h).
    """
    f32 = x.dtype == torch.float32
    B, H, W, Cx = x.shape
    cout, cin_w, kh, kw = w.shape
    cin = cin or cin_w
    if pad is None:
        pad = (kh // 2, kw // 2)
    if isinstance(pad, int):
        pad = (pad, pad)
    if out_hw is None:
        Ho = (H + 2 * pad[0] - kh) // stride + 1
        Wo = (W + 2 * pad[1] - kw) // stride + 1
    else:
        Ho, Wo = out_hw
    if out is None:
        out = torch.empty(B, Ho, Wo, cout, dtype=torch.float32 if (f32out or f32) else torch.bfloat16, device=x.device)
    wt, bt, kpad, cpad, w3 = packed if packed is not None else pack_weights(w, b, x.device, "fp32" if f32 else "bf16")
    pwd = {}
    if pw is not None:
        from ..engine.planner import pack_pw_weight_x3

        if not f32:
            raise ValueError("conv2d_nhwc: the functional fused pointwise path is fp32-only")
        w2, b2 = pw
        co2 = w2.shape[0]
        k2 = (cout + 31) // 32 * 32
        w2p = torch.frombuffer(bytearray(pack_pw_weight_x3(w2.detach().cpu().float(), k2)),
                               dtype=torch.int16).to(x.device)
        b2p = torch.zeros((co2 + 15) // 16 * 16)
        b2p[:co2] = b2.detach().float()
        b2p = b2p.to(x.device)
        out = torch.empty(B, Ho, Wo, co2, dtype=torch.float32, device=x.device)
        pwd = {"pw_w": _ptr(w2p), "pw_bias": _ptr(b2p), "pw_y": _ptr(out), "pw_ys": co2, "pw_cout": co2,
               "pw_kpad": k2, "pw_act": 0}
    skd = {}
    if 171 <= int(impl) < 180:  # split-K x3g: a workspace for the partial tiles (splits <= 8)
        ws = torch.empty(8 * B * Ho * Wo * cpad, dtype=torch.float32, device=x.device)
        skd = {"sk_ws": _ptr(ws), "sk_ws_bytes": ws.numel() * 4}
    native().conv2d({
        "x": _ptr(x, x_coff), "B": B, "H": H, "W": W, "xs": Cx, "Cin": cin,
        "w": _ptr(wt), "Kpad": kpad, "bias": _ptr(bt),
        "y": _ptr(out, out_coff), "Ho": Ho, "Wo": Wo, "ys": out.shape[-1], "Cout": cout, "Cout_pad": cpad,
        "KH": kh, "KW": kw, "stride": stride, "pad_t": pad[0], "pad_l": pad[1],
        "res": _ptr(res, res_coff), "rs": res.shape[-1] if res is not None else 0,
        "y2": _ptr(out2, out2_coff), "y2s": out2.shape[-1] if out2 is not None else 0,
        "act": ACT[act], "f32out": int(f32out), "bdev": _ptr(bdev), "stream": _stream(), "f32": int(f32),
        "impl": int(impl), "w3": _ptr(w3), **pwd, **skd,
    })
    if pw is not None:
        torch.cuda.synchronize(x.device)  # keep the packed 1x1 weights alive until the kernel ran
    return out


def dwconv3x3_nhwc(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, *, stride: int = 1, act="relu6",
                   bdev: torch.Tensor | None = None) -> torch.Tensor:
    B, H, W, C = x.shape
    f32 = x.dtype == torch.float32
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.empty(B, Ho, Wo, C, dtype=x.dtype, device=x.device)
    wt = w.detach().float().reshape(C, 9).t().contiguous().to(x.dtype).to(x.device)
    bt = b.detach().float().contiguous().to(x.device)
    native().dwconv3x3({"x": _ptr(x), "B": B, "H": H, "W": W, "xs": C, "C": C, "w": _ptr(wt), "bias": _ptr(bt),
                        "y": _ptr(y), "Ho": Ho, "Wo": Wo, "ys": C, "stride": stride, "act": ACT[act],
                        "bdev": _ptr(bdev), "stream": _stream(), "f32": int(f32)})
    return y


def ir_block_nhwc(x: torch.Tensor, expand, dw, project, *, stride: int, res: bool = False,
                  bdev: torch.Tensor | None = None, x_parts: int = 1, y_parts: int = 1) -> torch.Tensor:
    """Fused MobileNetV2 inverted residual (expand 1x1+ReLU6 -> dw3x3+ReLU6 -> project 1x1 [+x]).
    ``expand``/``dw``/``project`` are (weight, bias) pairs with BN folded; ``expand`` None for t=1.
    ``x_parts`` / ``y_parts`` (fp32 14x14 whole-map kernel): ``x`` holds x_parts partial sums of the input side by
    side on the channel axis; the result holds y_parts partial sums (hidden channels split over workgroups)."""
    from ..engine.planner import ir_x3_plan, pack_ir_weights, split_bf16x3

    B, H, W, Ct = x.shape
    C = Ct // x_parts
    f32 = x.dtype == torch.float32  # fp32 kernels (csrc/kernels/ir_f32.hip, ir_crop_f32.hip, ir_tile_x3.hip)
    pk = pack_ir_weights(expand, dw, project, C, k_align=16 if f32 else 32)
    x3w = 0
    if f32:
        x3w, inp_x3 = ir_x3_plan(H, W, stride, C, pk["hid_pad"], pk["oup_pad"], int(expand is not None))
        if x3w and inp_x3 != pk["inp_pad"]:
            pk = pack_ir_weights(expand, dw, project, C, k_align=32)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.empty(B, Ho, Wo, pk["oup"] * y_parts, dtype=x.dtype, device=x.device)
    mat = torch.float32 if f32 else torch.bfloat16
    dev = {k: (pk[k].to(mat) if k in ("we", "wd", "wp") else pk[k].float()).contiguous().to(x.device)
           for k in ("we", "be", "wd", "bd", "wp", "bp")}
    if x3w:  # the whole-map kernel reads pre-split [h|m|l] bf16 expand / project weights
        dev["we"] = split_bf16x3(pk["we"]).to(x.device)
        dev["wp"] = split_bf16x3(pk["wp"]).to(x.device)
    native().ir_block({"x": _ptr(x), "x_cs": Ct, "H": H, "W": W, "inp": C, "inp_pad": pk["inp_pad"],
                       "hid_pad": pk["hid_pad"], "oup": pk["oup"], "oup_pad": pk["oup_pad"], "stride": stride,
                       "expand": int(expand is not None), "res": int(res),
                       **{k: _ptr(v) for k, v in dev.items()}, "y": _ptr(y), "y_cs": pk["oup"] * y_parts, "Ho": Ho,
                       "Wo": Wo, "B": B, "bdev": _ptr(bdev), "stream": _stream(), "f32": int(f32), "x3w": x3w,
                       "x_parts": x_parts, "y_parts": y_parts})
    torch.cuda.synchronize(x.device)  # keep the packed weights alive until the kernel ran
    return y


def c3_x3_nhwc(x: torch.Tensor, cv12, bottleneck, cv3) -> torch.Tensor:
    """fp32 YOLOv5 C3 block at 160x160 geometry (C1 32, c_ 16, one bottleneck with shortcut) as one kernel
    (csrc/kernels/c3_x3.hip); ``cv12`` = (w [32, 32, 1, 1], b) of cv1|cv2 stacked, ``bottleneck`` =
    ((w1 [16, 16, 1, 1], b1), (w2 [16, 16, 3, 3], b2)), ``cv3`` = (w [32, 32, 1, 1], b); BN folded."""
    from ..engine.planner import split_bf16x3

    B, H, W, C = x.shape
    (w1, b1), (w2, b2) = bottleneck
    w2k = torch.zeros(16, 160)
    w2k[:, :144] = w2.detach().float().permute(0, 2, 3, 1).reshape(16, 144)
    dev = {"w12": split_bf16x3(cv12[0].reshape(32, 32)), "b12": cv12[1].float(),
           "wb1": split_bf16x3(w1.reshape(16, 16)), "bb1": b1.float(), "wb2": split_bf16x3(w2k), "bb2": b2.float(),
           "w3": split_bf16x3(cv3[0].reshape(32, 32)), "b3": cv3[1].float()}
    dev = {k: v.contiguous().to(x.device) for k, v in dev.items()}
    y = torch.empty(B, H, W, 32, dtype=torch.float32, device=x.device)
    native().c3_block({"x": _ptr(x), "xs": C, "B": B, "H": H, "W": W, "bdev": 0, "C1": 32, "CH": 16, "NB": 1,
                       "res": 1, **{k: _ptr(v) for k, v in dev.items()}, "y": _ptr(y), "ys": 32,
                       "stream": _stream(), "f32": 1})
    torch.cuda.synchronize(x.device)
    return y


def sppf_nhwc(buf: torch.Tensor, C: int) -> torch.Tensor:
    """In place: buf[..., C:4C] = cascaded 5x5 max pools of buf[..., :C]."""
    B, H, W, Ct = buf.shape
    native().sppf_pool({"buf": _ptr(buf), "B": B, "H": H, "W": W, "xs": Ct, "C": C, "stream": _stream(),
                        "f32": int(buf.dtype == torch.float32)})
    return buf


def image_meta_bytes(images: list[np.ndarray], T: int) -> tuple[bytes, np.ndarray]:
    """Pack images into one uint8 pool (256-B aligned) + ImageMeta records."""
    from ..processing.transforms import letterbox_geometry

    metas, chunks, off = [], [], 0
    for im in images:
        h, w = im.shape[:2]
        scale, nw, nh, pw, ph = letterbox_geometry(h, w, T)
        metas.append(IMAGE_META.pack(off, h, w, nw, nh, pw, ph, scale))
        data = np.ascontiguousarray(im, np.uint8).tobytes()
        pad = (-len(data)) % 256
        chunks.append(data + b"\0" * pad)
        off += len(data) + pad
    return b"".join(metas), np.frombuffer(b"".join(chunks), dtype=np.uint8)


def ctrl_tensor(n_images: int, device, n_crops: int = 0, crop_base: int = 0) -> torch.Tensor:
    c = torch.zeros(16, dtype=torch.int32)
    c[0], c[1], c[2] = n_images, n_crops, crop_base
    return c.to(device)


def letterbox_s2d(images: list[np.ndarray], T: int, device, dtype=torch.bfloat16) -> torch.Tensor:
    meta, pool = image_meta_bytes(images, T)
    meta_t = torch.frombuffer(bytearray(meta), dtype=torch.uint8).to(device)
    pool_t = torch.from_numpy(pool.copy()).to(device)
    ctrl = ctrl_tensor(len(images), device)
    out = torch.empty(len(images), T // 2, T // 2, 16, dtype=dtype, device=device)
    native().letterbox_s2d({"pool": _ptr(pool_t), "meta": _ptr(meta_t), "ctrl": _ptr(ctrl), "out": _ptr(out),
                            "B": len(images), "T": T, "stream": _stream(), "f32": int(dtype == torch.float32)})
    torch.cuda.current_stream().synchronize()
    return out


def s2d_to_nchw(x: torch.Tensor) -> torch.Tensor:
    """[B, h, w, 16] space-to-depth (12 live channels) -> [B, 3, 2h, 2w] fp32."""
    B, h, w, _ = x.shape
    y = x[..., :12].float().reshape(B, h, w, 2, 2, 3)  # p, q, c
    return y.permute(0, 5, 1, 3, 2, 4).reshape(B, 3, 2 * h, 2 * w)


def avgpool_nhwc(x: torch.Tensor) -> torch.Tensor:
    B, H, W, C = x.shape
    y = torch.empty(B, C, dtype=x.dtype, device=x.device)
    native().global_avgpool({"x": _ptr(x), "B": B, "HW": H * W, "C": C, "y": _ptr(y), "stream": _stream(),
                             "f32": int(x.dtype == torch.float32)})
    return y


def head_pool_nhwc(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, act: str | None = "relu6",
                   bdev: torch.Tensor | None = None) -> torch.Tensor:
    """mean over pixels of act(conv1x1(x, w) + b): [B,H,W,C] -> [B, N] (head_pool.hip); bf16 in/out, or fp32
    in/out (fp32-accurate triple-bf16-split kernel) for a float32 ``x``."""
    from ..engine.planner import ACT, pack_conv_weight

    B, H, W, C = x.shape
    N = w.shape[0]
    f32 = x.dtype == torch.float32
    wb, bb, kpad, npad = pack_conv_weight(w, b, "fp32" if f32 else "bf16")
    wd = torch.frombuffer(bytearray(wb), dtype=torch.float32 if f32 else torch.bfloat16).to(x.device)
    bd = torch.frombuffer(bytearray(bb), dtype=torch.float32).to(x.device)
    y = torch.empty(B, N, dtype=x.dtype, device=x.device)
    native().head_pool({"x": _ptr(x), "xs": C, "HW": H * W, "K": C, "w": _ptr(wd), "Kpad": kpad, "bias": _ptr(bd),
                        "N": N, "Npad": npad, "y": _ptr(y), "ys": N, "act": ACT[act], "B": B, "bdev": _ptr(bdev),
                        "stream": _stream(), "f32": int(f32)})
    torch.cuda.synchronize(x.device)  # keep the packed weights alive until the kernel ran
    return y


def topk_softmax(logits: torch.Tensor):
    """[B, N] fp32 -> (idx [B,5] int32, logit [B,5], prob [B,5])."""
    B, N = logits.shape
    out = torch.empty(B, 16, dtype=torch.int32, device=logits.device)
    native().topk_softmax({"logits": _ptr(logits), "B": B, "N": N, "ld": logits.stride(0), "out": _ptr(out),
                           "stream": _stream()})
    torch.cuda.current_stream().synchronize()
    o = out.cpu()
    return o[:, 0:5].clone(), o[:, 5:10].view(torch.float32).clone(), o[:, 10:15].view(torch.float32).clone()
