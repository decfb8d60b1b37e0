"""Exact-fp32 pipeline (csrc/kernels/conv_f32.hip + the fp32 instantiations of the
preprocessing / decode / pooling kernels) against plain PyTorch fp32/fp64 references.

The reference runs both networks as fp32 ONNX graphs (reference experiment.yaml:202,207,
220,225); these tests pin the MI355X fp32 path at that precision: kernel errors at the
fp32 rounding level, and the whole request pipeline equal to the fp32 torch/NumPy
reference pipeline (engine/reference.py) in detection counts, boxes, labels and logits.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from inference_arena_amd.ops import functional as AF

pytestmark = pytest.mark.gpu


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _act64(y, act):
    if act == "silu":
        return y * torch.sigmoid(y)
    if act == "relu6":
        return y.clamp(0.0, 6.0)
    return y


def _fp32_check(got, ref64, scale64, rel=2e-6):
    """|got - ref| <= rel * sum|x||w| (+ a denormal floor): fp32 products, fp32 accumulation."""
    err = (got.double().cpu() - ref64).abs()
    bound = rel * scale64 + 1e-30
    worst = (err / bound).max().item()
    assert worst <= 1.0, f"max error {err.max().item():.3g} is {worst:.2f}x the fp32 bound"


@pytest.mark.parametrize(
    "B,H,Cin,Cout,k,s,act,res,up",
    [
        (2, 20, 16, 16, 3, 1, "silu", False, False),    # s2d stem geometry (3x3 over 16 channels)
        (2, 40, 16, 32, 3, 2, "silu", False, False),    # 3x3 stride 2
        (3, 20, 32, 32, 3, 1, "silu", True, False),     # bottleneck with residual
        (2, 10, 64, 128, 1, 1, "silu", False, True),    # 1x1 with the 2x upsampled second store
        (4, 7, 160, 960, 1, 1, "relu6", False, False),  # MobileNet expand
        (4, 7, 960, 160, 1, 1, None, True, False),      # MobileNet project + residual
        (2, 10, 256, 144, 3, 1, "silu", False, False),  # detect head stacked cv2|cv3 (Cout 144: 9 tiles)
        (2, 20, 64, 80, 3, 1, "silu", False, False),    # Cout 80 (5 tiles)
        (5, 1, 1280, 1000, 1, 1, None, False, False),   # classifier FC as a 1x1 conv on a 1x1 map
    ],
)
def test_conv_f32_matches_fp64(device, B, H, Cin, Cout, k, s, act, res, up):
    g = torch.Generator().manual_seed(B * 100 + H + Cin + Cout)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g, dtype=torch.float64) * 0.1
    x32, w32, b32 = x.float(), w.float(), b.float()  # the kernel sees fp32 operands
    pad = k // 2
    ref = _act64(F.conv2d(x32.double(), w32.double(), b32.double(), stride=s, padding=pad), act)
    scale = F.conv2d(x32.double().abs(), w32.double().abs(), b32.double().abs(), stride=s, padding=pad)
    Ho = ref.shape[2]
    r = torch.randn(B, Cout, Ho, Ho, generator=g).float() if res else None
    if res:
        ref = ref + r.double()
        scale = scale + r.double().abs()
    out2 = torch.zeros(B, 2 * Ho, 2 * Ho, Cout, device=device) if up else None
    y = AF.conv2d_nhwc(_nhwc(x32).to(device), w32, b32, stride=s, act=act,
                       res=_nhwc(r).to(device) if res else None, out2=out2)
    torch.cuda.synchronize()
    assert y.dtype == torch.float32
    _fp32_check(y.permute(0, 3, 1, 2), ref, scale)
    if up:
        up_ref = y.repeat_interleave(2, 1).repeat_interleave(2, 2)
        assert torch.equal(out2, up_ref)


# x3 tile variants, split halo (auto/48/32), split stream (auto/32), FC, exact-fp32 stream — same fp32 bound
X3_IMPLS = [40 + v for v in range(12)] + [101, 102, 103, 104, 105, 106, 107, 108, 109, 110] + \
    [111 + v for v in range(20)]
X3G_IMPLS = [111 + v for v in range(20)]  # x3g: 32x32x16 MFMA GEMM over pre-split weights (gemm_x3.hip)
X3G_IMPLS += [171 + v for v in range(9)]  # ... split-K (partials in a workspace, summed in split order)


@pytest.mark.parametrize(
    "B,H,Cin,Cout,k,s,act,res,up",
    [
        (2, 40, 32, 64, 3, 2, "silu", False, False),    # detector 3x3 s2 (160 -> 80 geometry)
        (3, 20, 64, 128, 3, 2, "silu", False, False),   # 3x3 s2, Cin 64
        (2, 10, 128, 256, 3, 2, "silu", False, False),  # 3x3 s2, Cin 128, 8 N tiles of 32
        (3, 13, 128, 128, 1, 1, "silu", False, False),  # C3 1x1, partial pixel tiles
        (2, 9, 256, 128, 1, 1, "silu", False, True),    # neck 1x1 with the 2x upsampled copy
        (2, 11, 80, 80, 1, 1, "silu", False, False),    # Cin 80: a partial K chunk
        (5, 7, 160, 960, 1, 1, "relu6", False, False),  # MobileNet expand
        (5, 7, 960, 160, 1, 1, None, True, False),      # MobileNet project + residual
        (5, 7, 960, 320, 1, 1, None, False, False),     # last MobileNet project
        (2, 5, 512, 256, 1, 1, "silu", False, False),   # SPPF cv2 (K 512)
    ],
)
def test_conv_x3g_matches_fp64(device, B, H, Cin, Cout, k, s, act, res, up):
    """Every x3g variant (pre-split weights, activations split on staging) at the fp32 bound, incl. the
    residual and upsampled-copy epilogues."""
    g = torch.Generator().manual_seed(B * 1000 + H + Cin + Cout + k)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g, dtype=torch.float64) * 0.1
    x32, w32, b32 = x.float(), w.float(), b.float()
    pad = k // 2
    ref = _act64(F.conv2d(x32.double(), w32.double(), b32.double(), stride=s, padding=pad), act)
    scale = F.conv2d(x32.double().abs(), w32.double().abs(), b32.double().abs(), stride=s, padding=pad)
    Ho = ref.shape[2]
    r = torch.randn(B, Cout, Ho, Ho, generator=g).float() if res else None
    if res:
        ref = ref + r.double()
        scale = scale + r.double().abs()
    xd = _nhwc(x32).to(device)
    rd = _nhwc(r).to(device) if res else None
    packed = AF.pack_weights(w32, b32, device, "fp32")
    for impl in X3G_IMPLS:
        out2 = torch.full((B, 2 * Ho, 2 * Ho, Cout), float("nan"), device=device) if up else None
        y = AF.conv2d_nhwc(xd, w32, b32, stride=s, act=act, res=rd, packed=packed, impl=impl, out2=out2)
        torch.cuda.synchronize()
        _fp32_check(y.permute(0, 3, 1, 2), ref, scale)
        if up:
            want = y.permute(0, 3, 1, 2).repeat_interleave(2, 2).repeat_interleave(2, 3)
            assert torch.equal(out2.permute(0, 3, 1, 2), want), impl


def test_conv_x3g_channel_slices_and_live_batch(device):
    """Reads a channel slice of a wider buffer, stores into a channel slice, and honours the device-side live
    batch count (blocks past it leave the output untouched)."""
    g = torch.Generator().manual_seed(11)
    buf = torch.randn(4, 12, 12, 96, generator=g)
    w = torch.randn(64, 32, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    packed = AF.pack_weights(w, b, device, "fp32")
    ref = F.conv2d(buf[..., 32:64].permute(0, 3, 1, 2).double(), w.double(), b.double(), stride=2, padding=1)
    live = torch.tensor([3], dtype=torch.int32, device=device)
    for impl in X3G_IMPLS:
        out = torch.full((4, 6, 6, 128), 7.0, device=device)
        AF.conv2d_nhwc(buf.to(device), w, b, stride=2, act=None, x_coff=32, cin=32, out=out, out_coff=64,
                       packed=packed, impl=impl, bdev=live)
        torch.cuda.synchronize()
        got = out[:3, :, :, 64:].permute(0, 3, 1, 2).double().cpu()
        assert (got - ref[:3]).abs().max().item() < 1e-5, impl
        assert torch.all(out[:, :, :, :64] == 7.0) and torch.all(out[3] == 7.0), impl


X3HG_IMPLS = [131 + v for v in range(14)]  # x3hg: 3x3 s1 halo tiles, 32x32x16 MFMA, pre-split weights
X3HR_IMPLS = [151 + v for v in range(10)]  # x3hr: the same tiles, per-wave register weights (halo_x3g.hip)
X3HG_IMPLS = X3HG_IMPLS + X3HR_IMPLS


@pytest.mark.parametrize(
    "B,H,Cin,Cout,act,res,up,s",
    [
        (2, 20, 64, 144, "silu", False, False, 1),   # detect head stacked cv2|cv3 (Cout 144: a partial 160 tile)
        (2, 19, 80, 80, "silu", False, False, 1),    # Cin 80 (five 16-deep chunks), partial pixel tiles
        (3, 17, 32, 32, "silu", True, False, 1),     # C3 bottleneck 3x3 with residual
        (2, 12, 128, 64, None, False, True, 1),      # wide K, 2x upsampled copy, no activation
        (2, 9, 20, 48, "relu6", False, False, 1),    # Cin 20: a partial 16-channel chunk
    ],
)
def test_conv_x3hg_matches_fp64(device, B, H, Cin, Cout, act, res, up, s):
    """Every x3hg variant at the fp32 bound, incl. partial channel chunks / pixel tiles / channel tiles and
    the residual and upsampled-copy epilogues (csrc/kernels/halo_x3g.hip)."""
    g = torch.Generator().manual_seed(B * 977 + H + Cin + Cout)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g, dtype=torch.float64) * 0.1
    x32, w32, b32 = x.float(), w.float(), b.float()
    ref = _act64(F.conv2d(x32.double(), w32.double(), b32.double(), stride=s, padding=1), act)
    scale = F.conv2d(x32.double().abs(), w32.double().abs(), b32.double().abs(), stride=s, padding=1)
    Ho = ref.shape[2]
    r = torch.randn(B, Cout, Ho, Ho, generator=g).float() if res else None
    if res:
        ref = ref + r.double()
        scale = scale + r.double().abs()
    xd = _nhwc(x32).to(device)
    rd = _nhwc(r).to(device) if res else None
    packed = AF.pack_weights(w32, b32, device, "fp32")
    bad = []
    for impl in X3HG_IMPLS:
        out2 = torch.full((B, 2 * Ho, 2 * Ho, Cout), float("nan"), device=device) if up else None
        y = AF.conv2d_nhwc(xd, w32, b32, stride=s, act=act, res=rd, packed=packed, impl=impl, out2=out2)
        torch.cuda.synchronize()
        try:
            _fp32_check(y.permute(0, 3, 1, 2), ref, scale)
        except AssertionError as e:
            bad.append((impl, str(e)))
            continue
        if up:
            want = y.permute(0, 3, 1, 2).repeat_interleave(2, 2).repeat_interleave(2, 3)
            assert torch.equal(out2.permute(0, 3, 1, 2), want), impl
    assert not bad, bad


X3HG_PW_IMPLS = [145 + v for v in range(6)] + [161 + v for v in range(6)]  # x3hg / x3hr with the fused 1x1
X3HG_PW_IMPLS += [181, 182]  # x3hg-pw 8 x 8 pixel tiles on 2 waves (small buckets)


@pytest.mark.parametrize("B,H,Cin,C", [(2, 20, 64, 64), (2, 19, 80, 80), (3, 11, 144, 64)])
def test_conv_x3hg_fused_pointwise_matches_fp64(device, B, H, Cin, C):
    """3x3 (+ SiLU) -> 1x1 in one kernel (the 3x3 result never stored) at the fp32 bound of the composite:
    every variant whose channel tile fits (box branch 64 -> 64, cls branch 80 -> 80)."""
    g = torch.Generator().manual_seed(B * 31 + H + Cin + C)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64).float()
    w = (torch.randn(C, Cin, 3, 3, generator=g, dtype=torch.float64) / (Cin * 9) ** 0.5).float()
    b = (torch.randn(C, generator=g, dtype=torch.float64) * 0.1).float()
    w2 = (torch.randn(C, C, 1, 1, generator=g, dtype=torch.float64) / C ** 0.5).float()
    b2 = (torch.randn(C, generator=g, dtype=torch.float64) * 0.1).float()
    a = _act64(F.conv2d(x.double(), w.double(), b.double(), padding=1), "silu")
    ref = F.conv2d(a, w2.double(), b2.double())
    s1 = F.conv2d(x.double().abs(), w.double().abs(), b.double().abs(), padding=1)
    scale = F.conv2d(1.2 * s1 + a.abs(), w2.double().abs(), b2.double().abs())
    xd = _nhwc(x).to(device)
    packed = AF.pack_weights(w, b, device, "fp32")
    ran = 0
    for impl in [0] + X3HG_PW_IMPLS:
        try:
            y = AF.conv2d_nhwc(xd, w, b, act="silu", packed=packed, impl=impl, pw=(w2, b2))
        except RuntimeError:
            assert impl != 0, "the default fused-pointwise variant must take the detect-head shapes"
            continue
        torch.cuda.synchronize()
        assert y.shape == (B, H, H, C)
        _fp32_check(y.permute(0, 3, 1, 2), ref, scale)
        ran += 1
    assert ran >= 3


# x3hg variant -> the x3hr variant with the same tile (TW, WM, WN, TM, TN)
X3HR_SAME_TILE = {131: 151, 132: 152, 134: 153, 135: 154, 137: 155, 142: 156, 139: 157, 140: 158, 133: 159,
                  141: 160}


@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 20, 64, 144), (2, 19, 80, 80), (3, 13, 48, 64)])
def test_conv_x3hr_bit_identical_to_x3hg(device, B, H, Cin, Cout):
    """x3hr changes where the weights come from (registers, not an LDS stage), not the arithmetic: same tile, same
    products in the same order, so the outputs equal x3hg's bit for bit, plain and with the fused 1x1."""
    g = torch.Generator().manual_seed(B + H + Cin + Cout)
    x = torch.randn(B, H, H, Cin, generator=g).to(device)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    packed = AF.pack_weights(w, b, device, "fp32")
    for hg, hr in X3HR_SAME_TILE.items():
        y0 = AF.conv2d_nhwc(x, w, b, act="silu", packed=packed, impl=hg)
        y1 = AF.conv2d_nhwc(x, w, b, act="silu", packed=packed, impl=hr)
        torch.cuda.synchronize()
        assert torch.equal(y0, y1), (hg, hr)
    if Cout in (64, 80):
        w2 = torch.randn(Cout, Cout, 1, 1, generator=g) / Cout ** 0.5
        b2 = torch.randn(Cout, generator=g) * 0.1
        for v in range(6):
            try:
                y0 = AF.conv2d_nhwc(x, w, b, act="silu", packed=packed, impl=145 + v, pw=(w2, b2))
            except RuntimeError:
                continue
            y1 = AF.conv2d_nhwc(x, w, b, act="silu", packed=packed, impl=161 + v, pw=(w2, b2))
            torch.cuda.synchronize()
            assert torch.equal(y0, y1), v


def test_conv_x3hg_channel_slices_and_live_batch(device):
    """Channel-slice input and output views and the device-side live batch count."""
    g = torch.Generator().manual_seed(13)
    buf = torch.randn(4, 11, 11, 96, generator=g)
    w = torch.randn(64, 32, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g) * 0.1
    packed = AF.pack_weights(w, b, device, "fp32")
    ref = F.conv2d(buf[..., 32:64].permute(0, 3, 1, 2).double(), w.double(), b.double(), padding=1)
    live = torch.tensor([3], dtype=torch.int32, device=device)
    for impl in X3HG_IMPLS:
        out = torch.full((4, 11, 11, 128), 7.0, device=device)
        AF.conv2d_nhwc(buf.to(device), w, b, stride=1, act=None, x_coff=32, cin=32, out=out, out_coff=64,
                       packed=packed, impl=impl, bdev=live)
        torch.cuda.synchronize()
        got = out[:3, :, :, 64:].permute(0, 3, 1, 2).double().cpu()
        assert (got - ref[:3]).abs().max().item() < 1e-5, impl
        assert torch.all(out[:, :, :, :64] == 7.0) and torch.all(out[3] == 7.0), impl


@pytest.mark.parametrize(
    "B,H,Cin,Cout,k,s,act,res",
    [
        (2, 20, 32, 32, 3, 1, "silu", True),       # bottleneck 3x3 with residual
        (2, 24, 80, 80, 3, 1, "silu", False),      # Cin 80: a partial 32-channel chunk in the halo kernel
        (2, 20, 64, 144, 3, 1, "silu", False),     # detect head (Cout 144)
        (2, 40, 16, 32, 3, 2, "silu", False),      # 3x3 stride 2
        (2, 12, 16, 32, 2, 1, "relu6", False),     # 2x2 over a space-to-depth stem (MobileNetV2 stem)
        (2, 20, 16, 16, 3, 1, "silu", True),       # YOLO s2d stem 3x3 over 16 channels (+ residual)
        (4, 7, 160, 960, 1, 1, "relu6", False),    # MobileNet expand
        (4, 7, 960, 160, 1, 1, None, True),        # MobileNet project + residual
    ],
)
def test_conv_x3_split_matches_fp64(device, B, H, Cin, Cout, k, s, act, res):
    """The fp32-accurate triple-bf16-split kernels (bf16 matrix cores, six partial products) meet the same
    fp32 error bound as the exact-fp32 kernels, for every tile variant."""
    g = torch.Generator().manual_seed(B * 100 + H + Cin + Cout)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g, dtype=torch.float64) * 0.1
    x32, w32, b32 = x.float(), w.float(), b.float()
    pad = k // 2
    ref = _act64(F.conv2d(x32.double(), w32.double(), b32.double(), stride=s, padding=pad), act)
    scale = F.conv2d(x32.double().abs(), w32.double().abs(), b32.double().abs(), stride=s, padding=pad)
    Ho = ref.shape[2]
    r = torch.randn(B, Cout, Ho, Ho, generator=g).float() if res else None
    if res:
        ref = ref + r.double()
        scale = scale + r.double().abs()
    xd = _nhwc(x32).to(device)
    rd = _nhwc(r).to(device) if res else None
    packed = AF.pack_weights(w32, b32, device, "fp32")
    ran = 0
    for impl in X3_IMPLS:
        try:
            y = AF.conv2d_nhwc(xd, w32, b32, stride=s, act=act, res=rd, packed=packed, impl=impl)
        except RuntimeError as e:
            assert "eligible" in str(e), e  # split halo: 3x3 s1; stream: Cin % 8, K <= 192; FC: 1x1 map, K 1280
            continue
        torch.cuda.synchronize()
        _fp32_check(y.permute(0, 3, 1, 2), ref, scale)
        ran += 1
    assert ran >= 12


def test_conv_f32_channel_slices(device):
    """Reads channels [x_coff, x_coff + Cin) of a wider buffer and stores into a channel slice (concat)."""
    g = torch.Generator().manual_seed(7)
    buf = torch.randn(2, 12, 12, 96, generator=g)
    w = torch.randn(32, 48, 3, 3, generator=g) * 0.05
    b = torch.randn(32, generator=g) * 0.1
    out = torch.full((2, 12, 12, 64), 7.0, device=device)
    AF.conv2d_nhwc(buf.to(device), w, b, x_coff=16, cin=48, out=out, out_coff=32, act=None)
    torch.cuda.synchronize()
    ref = F.conv2d(buf[..., 16:64].permute(0, 3, 1, 2).double(), w.double(), b.double(), padding=1)
    o = out.cpu()
    assert torch.all(o[..., :32] == 7.0)  # untouched slice
    np.testing.assert_allclose(o[..., 32:].permute(0, 3, 1, 2).double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("stride,H", [(1, 14), (2, 28), (1, 7), (2, 112)])
def test_dwconv_f32(device, stride, H):
    g = torch.Generator().manual_seed(stride * 10 + H)
    C = 96
    x = torch.randn(3, C, H, H, generator=g)
    w = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(C, generator=g) * 0.1
    y = AF.dwconv3x3_nhwc(_nhwc(x).to(device), w, b, stride=stride, act="relu6")
    torch.cuda.synchronize()
    ref = F.relu6(F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=1, groups=C))
    np.testing.assert_allclose(y.permute(0, 3, 1, 2).double().cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


def test_sppf_f32_exact(device):
    g = torch.Generator().manual_seed(3)
    C = 128
    buf = torch.zeros(2, 20, 20, 4 * C)
    buf[..., :C] = torch.randn(2, 20, 20, C, generator=g)
    got = AF.sppf_nhwc(buf.to(device), C).cpu()
    x = buf[..., :C].permute(0, 3, 1, 2)
    y1 = F.max_pool2d(x, 5, 1, 2)
    y2 = F.max_pool2d(y1, 5, 1, 2)
    y3 = F.max_pool2d(y2, 5, 1, 2)
    for i, ref in enumerate((y1, y2, y3), start=1):
        assert torch.equal(got[..., i * C:(i + 1) * C], ref.permute(0, 2, 3, 1)), i


def test_letterbox_f32_equals_host(device):
    """Device letterbox in fp32 == the host reference preprocessor (uint8 rounding + /255), bit for bit."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.processing import YOLOPreprocessor

    imgs = synthetic_images(2, 5) + synthetic_images(1, 6, hw=(333, 500)) + synthetic_images(1, 7, hw=(640, 427))
    out = AF.letterbox_s2d(imgs, 640, device, dtype=torch.float32)
    got = AF.s2d_to_nchw(out.cpu())
    pre = YOLOPreprocessor()
    for i, im in enumerate(imgs):
        ref = torch.from_numpy(pre(im).tensor[0])
        assert torch.equal(got[i], ref), (i, (got[i] - ref).abs().max().item())


def test_avgpool_f32(device):
    x = torch.randn(5, 7, 7, 1280)
    y = AF.avgpool_nhwc(x.to(device)).cpu()
    np.testing.assert_allclose(y.numpy(), x.double().mean((1, 2)).numpy(), rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------------------- whole programs
def _iou(a, b):
    x1 = np.maximum(a[:, None, 0], b[None, :, 0])
    y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2])
    y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    bb = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + bb[None, :] - inter + 1e-9)


@pytest.fixture(scope="module")
def dense_models():
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    return make_yolo(0, cls_shift=-20.0), make_mobilenet(1)


def test_fp32_pipeline_matches_reference(dense_models, device):
    """The fp32 device pipeline equals the fp32 reference pipeline (torch CPU + host preprocessing +
    reference NMS): identical detection count per image, matched boxes with IoU > 0.99 and the same
    class, >= 99 % top-1 agreement and top-1 logit relative error < 1e-3."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.engine.reference import ReferencePipeline

    imgs = synthetic_images(10, 21) + synthetic_images(2, 22, hw=(333, 500)) + synthetic_images(2, 23, hw=(640, 427))
    pipe = GpuPipeline(*dense_models, device=0, buckets=[1, 8, 16], dtype="fp32")
    assert pipe.dtype == "fp32"
    got = pipe.infer(imgs)
    ref = ReferencePipeline(*dense_models, device="cpu")
    n_det = n_top1 = n_same_crop = 0
    rel = []
    for i, (im, g) in enumerate(zip(imgs, got)):
        r = ref(im)
        assert len(g) == len(r), f"image {i}: {len(g)} detections vs reference {len(r)}"
        if not len(r):
            continue
        iou = _iou(r.boxes, g.boxes)
        for j in range(len(r)):
            k = int(np.argmax(iou[j]))
            assert iou[j, k] > 0.99, (i, j, iou[j, k])
            assert g.classes[k] == r.classes[j]
            assert abs(float(g.scores[k]) - float(r.scores[j])) < 1e-4
            n_det += 1
            n_top1 += int(g.topk_idx[k, 0] == r.topk_idx[j, 0])
            # the crop is the int-truncated box (reference extract_crop): a box coordinate within fp32 rounding
            # of an integer may truncate one pixel apart, which is a different crop, not a precision error
            if np.array_equal(np.trunc(g.boxes[k]), np.trunc(r.boxes[j])):
                n_same_crop += 1
                rel.append(abs(float(g.topk_logit[k, 0]) - float(r.topk_logit[j, 0]))
                           / (abs(float(r.topk_logit[j, 0])) + 1e-6))
    assert n_det >= 20, n_det
    assert n_top1 >= 0.99 * n_det, (n_top1, n_det)
    assert n_same_crop >= 0.95 * n_det, (n_same_crop, n_det)
    assert max(rel) < 1e-3, max(rel)


def test_pipeline_stage_stamps(dense_models, device):
    """The program's wall-clock stamps (planner OP_STAMP): detection and classification device time per batch,
    both positive, together within the batch's event-timed gpu_ms (which adds H2D / D2H)."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    pipe = GpuPipeline(*dense_models, device=0, buckets=[8], dtype="fp32")
    imgs = synthetic_images(8, 91)
    pipe.ex.run(imgs)
    r = pipe.ex.run(imgs)
    assert r["detection_ms"] > 0 and r["classification_ms"] > 0
    assert r["detection_ms"] + r["classification_ms"] <= r["gpu_ms"] * 1.02 + 0.01
    assert r["detection_ms"] > r["classification_ms"] * 0.2  # YOLOv5nu is the larger share at 4 crops / image


def test_fp32_letterbox_stem_matches_unfused(dense_models, device, monkeypatch):
    """The fp32 stem conv sampling the letterboxed images itself (letterbox_conv, ARENA_F32_LB_STEM) vs the
    letterbox op + stem conv: the same stem activations (fp32 rounding) and the same results.  Covers
    unit-scale (640x480 / 640x427), bilinear (333x500) and padded images and a partial batch."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.engine.planner import BUF_POOL, OP_CONV, OP_LETTERBOX

    imgs = synthetic_images(3, 71) + synthetic_images(1, 72, hw=(333, 500)) + synthetic_images(1, 73, hw=(640, 427))
    monkeypatch.setenv("ARENA_F32_STEM_S2", "0")  # this test pins the letterbox-sampling stem conv alone
    monkeypatch.setenv("ARENA_F32_LB_STEM", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    monkeypatch.setenv("ARENA_F32_LB_STEM", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    assert any(int(op[0]) == OP_LETTERBOX for op in plain.program.ops)
    assert not any(int(op[0]) == OP_LETTERBOX for op in fused.program.ops)
    assert any(int(op[0]) == OP_CONV and int(op[1]) == BUF_POOL for op in fused.program.ops)
    a, b = plain.infer(imgs), fused.infer(imgs)
    for i in range(len(imgs)):
        x1, x2 = plain.read_buffer("b0", 8, i), fused.read_buffer("b0", 8, i)
        np.testing.assert_allclose(x2, x1, rtol=1e-5, atol=1e-5)
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, rtol=2e-5, atol=5e-3)
            np.testing.assert_array_equal(y.topk_idx[:, 0], x.topk_idx[:, 0])


@pytest.mark.parametrize("th", ["4", "8"])
def test_fp32_stem_s2_fused_matches_unfused(dense_models, device, monkeypatch, th):
    """letterbox + stem + 3x3 s2 conv in one kernel (csrc/kernels/stem_x3.hip, ARENA_F32_STEM_S2; both tile
    heights) vs the letterbox-sampling stem conv + a separate s2 conv: the same 160x160x32 map to fp32 rounding
    and the same results, over unit-scale, bilinear and padded images and a partial batch."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.engine.planner import OP_STEMFUSED

    imgs = synthetic_images(3, 81) + synthetic_images(1, 82, hw=(333, 500)) + synthetic_images(1, 83, hw=(640, 427))
    monkeypatch.setenv("ARENA_STEM_X3_TH", th)
    monkeypatch.setenv("ARENA_F32_STEM_S2", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    monkeypatch.setenv("ARENA_F32_STEM_S2", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    assert not any(int(op[0]) == OP_STEMFUSED for op in plain.program.ops)
    assert any(int(op[0]) == OP_STEMFUSED for op in fused.program.ops)
    a, b = plain.infer(imgs), fused.infer(imgs)
    for i in range(len(imgs)):
        x1, x2 = plain.read_buffer("b1", 8, i), fused.read_buffer("b1", 8, i)
        np.testing.assert_allclose(x2, x1, rtol=1e-5, atol=1e-5)
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, rtol=2e-5, atol=5e-3)
            np.testing.assert_array_equal(y.topk_idx[:, 0], x.topk_idx[:, 0])


def test_fp32_stem_block1_fused_matches_unfused(dense_models, device, monkeypatch):
    """crop gather + s2d stem conv + MobileNetV2 block 1 in one kernel (ARENA_F32_STEM_IR, ir_f32.hip stem mode)
    vs the crop-gather op + stem conv + block-1 kernel: the same block-1 output for every crop (fp32 rounding:
    the stem sums run on the same fp32 MFMA, the depthwise / project code is shared) and the same results."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.engine.planner import OP_CROPGATHER

    imgs = synthetic_images(5, 81) + synthetic_images(1, 82, hw=(333, 500))
    monkeypatch.setenv("ARENA_F32_STEM_IR", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    monkeypatch.setenv("ARENA_F32_STEM_IR", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="fp32")
    assert any(int(op[0]) == OP_CROPGATHER for op in plain.program.ops)
    assert not any(int(op[0]) == OP_CROPGATHER for op in fused.program.ops)
    a, b = plain.infer(imgs), fused.infer(imgs)
    n_crops = sum(len(x) for x in a)
    assert n_crops >= 5
    for i in range(n_crops):
        x1, x2 = plain.read_buffer("m0.out", 8, i), fused.read_buffer("m0.out", 8, i)
        np.testing.assert_allclose(x2, x1, rtol=1e-5, atol=2e-5)
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            np.testing.assert_array_equal(y.topk_idx, x.topk_idx)
            np.testing.assert_allclose(y.topk_logit, x.topk_logit, rtol=1e-5, atol=1e-5)


def test_fp32_tensor_models_match_torch(models, device):
    """Reference tensor contracts in fp32: yolov5n [3,640,640] -> [84,8400], mobilenetv2 -> [1000]."""
    from inference_arena_amd.engine.pipeline import GpuTensorModel

    yolo, mnet = models
    g = torch.Generator().manual_seed(11)
    x = torch.rand(2, 3, 640, 640, generator=g)
    tm = GpuTensorModel.yolo(yolo, device=0, buckets=[2], dtype="fp32")
    got = torch.from_numpy(tm.infer(x.numpy()))
    with torch.no_grad():
        ref = yolo.eval()(x).float()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-3, atol=2e-3)
    c = torch.randn(3, 3, 224, 224, generator=g)
    cm = GpuTensorModel.mobilenet(mnet, device=0, buckets=[4], dtype="fp32")
    got = cm.infer(c.numpy())
    with torch.no_grad():
        ref = mnet.eval()(c).float().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-3 * np.abs(ref).max())


def test_fp32_split_programs_match_pipeline(dense_models, device):
    """Detector-only and classifier-only fp32 programs (microservices arm) agree with the fused fp32 program."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuClassifier, GpuDetector, GpuPipeline
    from inference_arena_amd.processing import extract_crop

    yolo, mnet = dense_models
    imgs = synthetic_images(4, 31)
    full = GpuPipeline(yolo, mnet, device=0, buckets=[4], dtype="fp32").infer(imgs)
    det = GpuDetector(yolo, device=0, buckets=[4], dtype="fp32").infer(imgs)
    cls = GpuClassifier(mnet, device=0, buckets=[16], dtype="fp32")
    for a, d, im in zip(full, det, imgs):
        assert len(a) == len(d)
        np.testing.assert_allclose(a.boxes, d.boxes, atol=1e-3)
        if len(a):
            crops = [extract_crop(im, np.concatenate([bx, [0.0, 0.0]])) for bx in a.boxes]
            out = cls.infer(crops)
            assert [int(o[0][0]) for o in out] == [int(t) for t in a.topk_idx[:, 0]]


def _ir_ref64(x, expand, dw, project, stride, res):
    h = x.double()
    if expand is not None:
        h = F.conv2d(h, expand[0].double(), expand[1].double()).clamp(0, 6)
    C = dw[0].shape[0]
    h = F.conv2d(h, dw[0].double(), dw[1].double(), stride=stride, padding=1, groups=C).clamp(0, 6)
    y = F.conv2d(h, project[0].double(), project[1].double())
    return y + x.double() if res else y


@pytest.mark.parametrize("inp,hid,oup,stride,H,res", [
    (32, 32, 16, 1, 40, False),    # t = 1 block (no expand), MobileNetV2 block 1 geometry
    (16, 96, 24, 2, 37, False),    # block 2: 16 -> 24, stride 2, odd size (ir_f32 either way)
    (32, 96, 24, 2, 37, False),    # stride 2 with a full 32-channel input (the x3 tile kernel)
    (24, 144, 24, 1, 28, True),    # block 3 (hid 144 -> 160 padded chunks), residual
    (24, 144, 24, 1, 56, True),    # block 3 at its own size (register-resident kernel, 7-row strips)
    (32, 192, 32, 1, 30, False),   # stride 1, a map that is no multiple of the 14-column strips
    (24, 144, 32, 2, 28, False),   # block 4
    (32, 192, 32, 1, 28, True),    # block 5/6
    (32, 192, 64, 2, 28, False),   # block 7 (4 output tiles of 16)
    # whole-map x3 kernel (csrc/kernels/ir_crop_f32.hip)
    (64, 384, 64, 1, 14, True),    # blocks 8-10
    (64, 384, 96, 1, 14, False),   # block 11
    (96, 576, 96, 1, 14, True),    # blocks 12-13
    (96, 576, 160, 2, 14, False),  # block 14 (14 -> 7)
    (160, 960, 160, 1, 7, True),   # blocks 15-16
    (160, 960, 320, 1, 7, False),  # block 17
])
@pytest.mark.parametrize("x3t", ["1", "0"])  # >= 28x28 expanding blocks: tiled x3 kernel / exact-fp32 ir_f32
def test_ir_block_f32_matches_fp64(device, inp, hid, oup, stride, H, res, x3t, monkeypatch, request):
    if H <= 14:  # the whole-map kernel (ARENA_IRC_F32=auto: the planner's default for these blocks); forced on here
        # ARENA_IR_X3T does not apply to it: the "0" slot runs the 14x14 kernel with four row bands per crop
        if x3t == "0" and H != 14:
            pytest.skip("one row-band layout at 7x7")
        monkeypatch.setenv("ARENA_IRC_F32", "1")
        from inference_arena_amd.ops import native

        native().set_irx_parts(4 if x3t == "0" else 2)
        request.addfinalizer(lambda: native().set_irx_parts(-1))
    monkeypatch.setenv("ARENA_IR_X3T", x3t)
    g = torch.Generator().manual_seed(inp * 7 + hid + stride)
    x = torch.randn(3, inp, H, H, generator=g)
    expand = None if hid == inp else (torch.randn(hid, inp, 1, 1, generator=g) / inp ** 0.5,
                                      torch.randn(hid, generator=g) * 0.1)
    dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
    project = (torch.randn(oup, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(oup, generator=g) * 0.1)
    y = AF.ir_block_nhwc(_nhwc(x).to(device), expand, dw, project, stride=stride, res=res)
    ref = _ir_ref64(x, expand, dw, project, stride, res)
    got = y.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs().max().item()
    assert err < 2e-5 * (1.0 + ref.abs().max().item()), err


@pytest.mark.parametrize("parts,crops", [(2, 5), (3, 5), (6, 5), (6, 40)])
@pytest.mark.parametrize("bands", [2, 4])
def test_ir_block_f32_hidden_slices_chain(device, parts, crops, bands, request):
    """Hidden-sliced 14x14 blocks (IrParams.x_parts / y_parts): block A writes its partial sums, block B adds
    them while loading its input (and for its residual) and writes one tensor — equal to the fp64 chain.  Crop
    capacities > 32 use at most set_irx_slices_big of the planned parts (3 here), on both sides."""
    from inference_arena_amd.ops import native

    native().set_irx_parts(bands)
    native().set_irx_slices_big(3)
    request.addfinalizer(lambda: (native().set_irx_parts(-1), native().set_irx_slices_big(-1)))
    eff = min(parts, 3) if crops > 32 else parts
    g = torch.Generator().manual_seed(parts * 11 + bands)
    blocks = []
    for inp, hid, oup in ((64, 384, 96), (96, 576, 96)):
        blocks.append(((torch.randn(hid, inp, 1, 1, generator=g) / inp ** 0.5, torch.randn(hid, generator=g) * 0.1),
                       (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1),
                       (torch.randn(oup, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(oup, generator=g) * 0.1)))
    x = torch.randn(crops, 64, 14, 14, generator=g)
    mid = AF.ir_block_nhwc(_nhwc(x).to(device), *blocks[0], stride=1, res=False, y_parts=parts)
    assert mid.shape[-1] == 96 * parts
    y = AF.ir_block_nhwc(mid, *blocks[1], stride=1, res=True, x_parts=parts)
    r0 = _ir_ref64(x, *blocks[0], 1, False)
    ref = _ir_ref64(r0.float(), *blocks[1], 1, True)
    got = y.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs().max().item()
    assert err < 2e-5 * (1.0 + ref.abs().max().item()), err
    summed = mid.reshape(crops, 14, 14, parts, 96)[..., :eff, :].double().sum(3).permute(0, 3, 1, 2).cpu()
    assert (summed - r0).abs().max().item() < 2e-5 * (1.0 + r0.abs().max().item())


@pytest.mark.parametrize("parts", [1, 3, 5])
def test_ir_block_f32_hidden_slices_tail(device, parts, monkeypatch):
    """The 14 -> 7 block and the 7x7 blocks on the whole-map kernel with hidden slices (ARENA_IRX_TAIL): one row
    band per crop at 7x7, partial sums from block 14 through block 16 into block 17's plain output."""
    monkeypatch.setenv("ARENA_IRC_F32", "1")  # the whole-map kernel for every 14x14 / 7x7 block
    g = torch.Generator().manual_seed(parts + 70)

    def blk(inp, hid, oup):
        return ((torch.randn(hid, inp, 1, 1, generator=g) / inp ** 0.5, torch.randn(hid, generator=g) * 0.1),
                (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1),
                (torch.randn(oup, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(oup, generator=g) * 0.1))

    b14, b15, b17 = blk(96, 576, 160), blk(160, 960, 160), blk(160, 960, 320)
    x = torch.randn(6, 96, 14, 14, generator=g)
    a = AF.ir_block_nhwc(_nhwc(x).to(device), *b14, stride=2, res=False, y_parts=parts)
    c = AF.ir_block_nhwc(a, *b15, stride=1, res=True, x_parts=parts, y_parts=parts)
    y = AF.ir_block_nhwc(c, *b17, stride=1, res=False, x_parts=parts)
    r14 = _ir_ref64(x, *b14, 2, False)
    r15 = _ir_ref64(r14.float(), *b15, 1, True)
    ref = _ir_ref64(r15.float(), *b17, 1, False)
    got = y.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs().max().item()
    assert err < 2e-5 * (1.0 + ref.abs().max().item()), err


@pytest.mark.parametrize("B,H,W", [(2, 24, 48), (1, 8, 16), (3, 16, 32)])
def test_c3_x3_matches_fp64(device, B, H, W):
    """The fp32 C3 block kernel (csrc/kernels/c3_x3.hip: cv1|cv2, bottleneck 1x1 + 3x3 + shortcut, cv3, all in
    one workgroup per 8 x 16 tile with a recomputed halo) against the four convs in fp64."""
    g = torch.Generator().manual_seed(B * 100 + H + W)
    x = torch.randn(B, 32, H, W, generator=g)
    cv12 = (torch.randn(32, 32, 1, 1, generator=g) / 32 ** 0.5, torch.randn(32, generator=g) * 0.1)
    bn = ((torch.randn(16, 16, 1, 1, generator=g) / 4, torch.randn(16, generator=g) * 0.1),
          (torch.randn(16, 16, 3, 3, generator=g) / 12, torch.randn(16, generator=g) * 0.1))
    cv3 = (torch.randn(32, 32, 1, 1, generator=g) / 32 ** 0.5, torch.randn(32, generator=g) * 0.1)
    y = AF.c3_x3_nhwc(_nhwc(x).to(device), cv12, bn, cv3)
    silu = lambda t: t * torch.sigmoid(t)  # noqa: E731
    d = lambda t: t.double()  # noqa: E731
    T = silu(F.conv2d(d(x), d(cv12[0]), d(cv12[1])))
    U = silu(F.conv2d(T[:, :16], d(bn[0][0]), d(bn[0][1])))
    T1 = T[:, :16] + silu(F.conv2d(U, d(bn[1][0]), d(bn[1][1]), padding=1))
    ref = silu(F.conv2d(torch.cat([T1, T[:, 16:]], 1), d(cv3[0]), d(cv3[1])))
    got = y.permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs().max().item()
    assert err < 2e-5 * (1.0 + ref.abs().max().item()), err


def test_fp32_fused_c3_program_matches_unfused(dense_models, device, monkeypatch):
    """fp32 pipeline with the 160x160 C3 block as one kernel vs the four-conv program: the block output at the
    fp32 level and identical detections / classifications."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(3, 51) + synthetic_images(1, 52, hw=(333, 500))
    monkeypatch.setenv("ARENA_FUSE_C3_F32", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="fp32")
    monkeypatch.setenv("ARENA_FUSE_C3_F32", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="fp32")
    assert sum(1 for op in fused.program.ops if int(op[0]) == 16) == 1
    assert sum(1 for op in plain.program.ops if int(op[0]) == 16) == 0
    a, b = plain.infer(imgs), fused.infer(imgs)
    for i in range(len(imgs)):
        x, y = plain.read_buffer("b2", 4, i), fused.read_buffer("b2", 4, i)
        np.testing.assert_allclose(y, x, rtol=0, atol=2e-5 * (1.0 + np.abs(x).max()))
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, atol=1e-2)
            assert [int(t) for t in x.topk_idx[:, 0]] == [int(t) for t in y.topk_idx[:, 0]]


def test_fp32_program_fuses_the_high_resolution_blocks():
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models

    p = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype="fp32")
    ir = [o for o in p.ops if int(o[0]) == 14]
    # block 1 fused with crop gather + stem (ir_f32.hip stem mode), >= 28x28: the tiled x3 kernel
    # (ir_tile_x3.hip, split-plane weights), stride-1 14x14: the x3 whole-map kernel (ir_crop_f32.hip);
    # 14 -> 7 and 7x7 blocks run unfused
    assert [(int(o[4]), int(o[26]), int(o[31])) for o in ir] == \
        [(112, 1, 1), (112, 0, 0), (56, 1, 0), (56, 1, 0), (28, 1, 0), (28, 1, 0), (28, 1, 0)] + [(14, 1, 0)] * 6
    assert all(int(o[7]) % 32 == 0 for o in ir if int(o[26]))  # x3 kernels step K by 32
    assert not [o for o in p.ops if int(o[0]) == 9]  # no separate crop gather
    assert all(int(o[47]) == 1 for o in p.ops)


@pytest.mark.parametrize("B,HW", [(5, 49), (3, 64), (2, 1)])
def test_head_pool_f32_matches_fp64(device, B, HW):
    """MobileNetV2 head conv (320 -> 1280) + ReLU6 + global average pool in one fp32-accurate kernel."""
    g = torch.Generator().manual_seed(B * 7 + HW)
    H = int(round(HW ** 0.5)) if int(round(HW ** 0.5)) ** 2 == HW else 1
    W = HW // H
    x = torch.randn(B, 320, H, W, generator=g)
    w = torch.randn(1280, 320, 1, 1, generator=g) / 320 ** 0.5
    b = torch.randn(1280, generator=g) * 0.1
    y = AF.head_pool_nhwc(_nhwc(x).to(device), w, b, "relu6")
    ref = F.conv2d(x.double(), w.double(), b.double()).clamp(0, 6).mean(dim=(2, 3))
    scale = F.conv2d(x.double().abs(), w.double().abs(), b.double().abs()).mean(dim=(2, 3))
    _fp32_check(y.double().cpu(), ref, scale, rel=4e-6)


