"""HIP kernels vs plain PyTorch fp32 references of the same op (MI355X only)."""
from __future__ import annotations

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from inference_arena_amd.ops import functional as AF
from inference_arena_amd.ops import native

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).float()


def _ref_conv(x_nhwc, w, b, stride, pad, act, res=None):
    y = F.conv2d(_nchw(x_nhwc).float(), _bf(w), b.float(), stride=stride, padding=pad)
    if act == "silu":
        y = F.silu(y)
    elif act == "relu6":
        y = F.relu6(y)
    if res is not None:
        y = y + _nchw(res).float()
    return y


def _check(got, ref, rtol=2e-2, atol=2e-2):
    err = (got.float() - ref.float()).abs()
    tol = atol + rtol * ref.float().abs()
    bad = (err > tol).float().mean().item()
    assert bad < 1e-3, f"{bad*100:.3f}% elements out of tolerance; max err {err.max().item():.4g}"


def test_native_loaded():
    C = native()
    assert C.SIZEOF_IMAGE_META == 48 and C.SIZEOF_CANDIDATE == 32 and C.SIZEOF_TOPK == 64


@pytest.fixture(params=[2, 1, 3], ids=["lds", "direct", "igemm"])
def conv_impl(request):
    C = native()
    old = C.get_conv_impl()
    C.set_conv_impl(request.param)
    yield request.param
    C.set_conv_impl(old)


@pytest.mark.parametrize(
    "B,H,Cin,Cout,k,s,act",
    [
        (2, 40, 32, 64, 3, 1, "silu"),
        (2, 40, 64, 128, 3, 2, "silu"),
        (1, 80, 16, 32, 3, 2, "silu"),  # Cin=16: k-groups straddle taps
        (3, 20, 256, 128, 1, 1, "silu"),
        (2, 28, 32, 144, 1, 1, "relu6"),  # 9 channel tiles (WC=3)
        (1, 20, 80, 80, 3, 1, "silu"),  # Cin=80, Cout=80 (WC=5)
        (2, 14, 96, 24, 1, 1, None),
        (1, 7, 320, 1280, 1, 1, "relu6"),
        (3, 20, 128, 64, 3, 2, "silu"),  # stride-2 tile with a partial column tile
        (2, 27, 64, 48, 3, 1, None),  # odd spatial size, 3 channel tiles
        (1, 20, 256, 144, 3, 1, "silu"),  # 8 input-channel slices
    ],
)
def test_conv_matches_torch(device, conv_impl, B, H, Cin, Cout, k, s, act):
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + Cin)
    x = torch.randn(B, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, generator=g) * 0.1
    xn = _nhwc(x).to(torch.bfloat16).to(device)
    y = AF.conv2d_nhwc(xn, w, b, stride=s, act=act)
    ref = _ref_conv(xn.cpu(), w, b, s, k // 2, act)
    _check(_nchw(y.cpu()), ref)


def test_conv_slices_residual_upsample(device, conv_impl):
    g = torch.Generator().manual_seed(7)
    B, H, Cbuf, Cin, Cout = 2, 20, 96, 32, 48
    buf = torch.randn(B, H, H, Cbuf, generator=g).to(torch.bfloat16).to(device)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    b = torch.randn(Cout, generator=g) * 0.1
    out = torch.zeros(B, H, H, 128, dtype=torch.bfloat16, device=device)
    res_buf = torch.randn(B, H, H, 64, generator=g).to(torch.bfloat16).to(device)
    up = torch.zeros(B, 2 * H, 2 * H, 64, dtype=torch.bfloat16, device=device)
    AF.conv2d_nhwc(buf, w, b, act="silu", x_coff=16, cin=Cin, out=out, out_coff=64, res=res_buf, res_coff=8,
                   out2=up, out2_coff=8)
    torch.cuda.synchronize()
    xs = buf.cpu()[..., 16:16 + Cin]
    ref = _ref_conv(xs, w, b, 1, 1, "silu", res=res_buf.cpu()[..., 8:8 + Cout])
    _check(_nchw(out.cpu()[..., 64:64 + Cout]), ref)
    assert out.cpu()[..., :64].abs().sum() == 0 and out.cpu()[..., 64 + Cout:].abs().sum() == 0
    upref = F.interpolate(_nchw(out.cpu()[..., 64:64 + Cout]), scale_factor=2, mode="nearest")
    assert torch.equal(_nchw(up.cpu()[..., 8:8 + Cout]), upref)


def test_conv_fp32_out_and_live_batch(device, conv_impl):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(6, 1, 1, 1280, generator=g).to(torch.bfloat16).to(device)
    w = torch.randn(1000, 1280, 1, 1, generator=g) / np.sqrt(1280)
    b = torch.randn(1000, generator=g)
    out = torch.full((6, 1, 1, 1000), -7.0, dtype=torch.float32, device=device)
    bdev = torch.tensor([4], dtype=torch.int32, device=device)
    AF.conv2d_nhwc(x, w, b, act=None, f32out=True, out=out, bdev=bdev)
    torch.cuda.synchronize()
    ref = x.cpu().float().reshape(6, 1280) @ _bf(w).reshape(1000, 1280).t() + b
    _check(out.cpu().reshape(6, 1000)[:4], ref[:4], rtol=1e-2, atol=1e-2)
    assert torch.all(out.cpu()[4:] == -7.0), "rows past the live batch must not be written"


def test_stem_s2d_equivalence(device, conv_impl):
    from inference_arena_amd.engine.plans import s2d_stem_3x3, s2d_stem_6x6

    g = torch.Generator().manual_seed(11)
    img = torch.rand(2, 3, 64, 64, generator=g)
    s2d = img.reshape(2, 3, 32, 2, 32, 2).permute(0, 2, 4, 3, 5, 1).reshape(2, 32, 32, 12)
    s2d = torch.cat([s2d, torch.zeros(2, 32, 32, 4)], -1).to(torch.bfloat16)
    xin = s2d.to(device)
    w6 = torch.randn(16, 3, 6, 6, generator=g) * 0.2
    b = torch.zeros(16)
    y = AF.conv2d_nhwc(xin, s2d_stem_6x6(w6), b, act=None)
    ref = F.conv2d(_bf(img), _bf(w6), None, stride=2, padding=2)
    _check(_nchw(y.cpu()), ref)
    w3 = torch.randn(32, 3, 3, 3, generator=g) * 0.2
    y3 = AF.conv2d_nhwc(xin, s2d_stem_3x3(w3), torch.zeros(32), pad=(1, 1), act=None, out_hw=(32, 32))
    ref3 = F.conv2d(_bf(img), _bf(w3), None, stride=2, padding=1)
    _check(_nchw(y3.cpu()), ref3)


@pytest.mark.parametrize("C,H,s", [(96, 56, 2), (144, 28, 1), (960, 7, 1), (32, 112, 1)])
def test_dwconv_matches_torch(device, C, H, s):
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(2, C, H, H, generator=g)
    w = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(C, generator=g) * 0.1
    xn = _nhwc(x).to(torch.bfloat16).to(device)
    y = AF.dwconv3x3_nhwc(xn, w, b, stride=s, act="relu6")
    ref = F.relu6(F.conv2d(_nchw(xn.cpu()), _bf(w), b, stride=s, padding=1, groups=C))
    _check(_nchw(y.cpu()), ref)


def test_sppf_matches_torch(device):
    g = torch.Generator().manual_seed(5)
    C = 128
    buf = torch.zeros(2, 20, 20, 4 * C, dtype=torch.bfloat16)
    buf[..., :C] = torch.randn(2, 20, 20, C, generator=g).to(torch.bfloat16)
    d = buf.to(device)
    AF.sppf_nhwc(d, C)
    torch.cuda.synchronize()
    x = _nchw(buf[..., :C])
    y1 = F.max_pool2d(x, 5, 1, 2)
    y2 = F.max_pool2d(y1, 5, 1, 2)
    y3 = F.max_pool2d(y2, 5, 1, 2)
    got = _nchw(d.cpu())
    for i, ref in enumerate((y1, y2, y3)):
        assert torch.equal(got[:, (i + 1) * C:(i + 2) * C], ref)


def test_letterbox_matches_host(device):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.processing import letterbox

    imgs = synthetic_images(3, 5) + [np.random.default_rng(0).integers(0, 255, (300, 1000, 3), dtype=np.uint8)]
    out = AF.letterbox_s2d(imgs, 640, device)
    got = AF.s2d_to_nchw(out.cpu())
    for i, im in enumerate(imgs):
        ref = torch.from_numpy(letterbox(im, 640)[0].astype(np.float32).transpose(2, 0, 1) / 255.0)
        err = (got[i] - ref).abs()
        # bf16 storage (~3 significant digits) + at most one uint8 rounding step
        assert (err <= 1.0 / 255 + 4e-3).float().mean() > 0.999, err.max()
        assert err.max() < 3.0 / 255 + 4e-3


def test_topk_and_avgpool(device):
    g = torch.Generator().manual_seed(9)
    logits = torch.randn(37, 1000, generator=g) * 3
    idx, lg, pr = AF.topk_softmax(logits.to(device))
    ref_v, ref_i = torch.topk(logits, 5, dim=1)
    assert torch.equal(idx.long(), ref_i)
    assert torch.allclose(lg, ref_v)
    assert torch.allclose(pr, torch.softmax(logits, 1).gather(1, ref_i), rtol=1e-4, atol=1e-6)
    # ties resolve to the lowest index (register path, N <= 1024) and the streaming path (N > 1024)
    for N in (1000, 77, 1500):
        t = torch.randint(0, 6, (9, N), generator=g).float()
        idx, lg, _ = AF.topk_softmax(t.to(device))
        order = np.lexsort((np.arange(N)[None, :].repeat(9, 0), -t.numpy()), axis=1)[:, :5]
        assert np.array_equal(idx.cpu().numpy(), order), N
        assert torch.equal(lg.cpu(), t.gather(1, torch.from_numpy(order)))
    x = torch.randn(5, 7, 7, 1280, generator=g).to(torch.bfloat16)
    y = AF.avgpool_nhwc(x.to(device))
    torch.cuda.synchronize()
    _check(y.cpu().float(), x.float().mean((1, 2)), rtol=1e-2, atol=1e-2)


def _ref_ir(x_nhwc, expand, dw, project, stride, res):
    """fp32 torch reference of one inverted residual on bf16-rounded operands."""
    x = _nchw(x_nhwc).float()
    h = x
    if expand is not None:
        h = F.relu6(F.conv2d(h, _bf(expand[0]), expand[1].float()))
        h = _bf(h)  # the kernel stores the expanded tile as bf16
    hid = dw[0].shape[0]
    h = F.relu6(F.conv2d(h, _bf(dw[0]), dw[1].float(), stride=stride, padding=1, groups=hid))
    h = _bf(h)
    y = F.conv2d(h, _bf(project[0]), project[1].float())
    return y + x if res else y


@pytest.mark.parametrize(
    "B,H,inp,hid,oup,s,res",
    [
        (2, 112, 32, 32, 16, 1, False),   # block 1: no expand
        (2, 112, 16, 96, 24, 2, False),   # block 2: 112 -> 56
        (2, 56, 24, 144, 24, 1, True),    # hidden 144 padded to 160
        (1, 56, 24, 144, 32, 2, False),
        (2, 28, 32, 192, 32, 1, True),
        (1, 28, 32, 192, 64, 2, False),
        (3, 14, 64, 384, 96, 1, False),
        (1, 14, 96, 576, 160, 2, False),
        (2, 7, 160, 960, 160, 1, True),
        (2, 7, 160, 960, 320, 1, False),
        (1, 20, 24, 144, 24, 1, True),    # partial 8x8 tiles are not used at 20 -> 7x7 tiles, partial edge
    ],
)
def test_ir_block_matches_torch(device, B, H, inp, hid, oup, s, res):
    g = torch.Generator().manual_seed(H * 100 + inp + oup)
    x = (torch.rand(B, inp, H, H, generator=g) * 2).to(torch.bfloat16)
    expand = None if hid == inp and H == 112 and inp == 32 else (
        torch.randn(hid, inp, 1, 1, generator=g) / np.sqrt(inp), torch.randn(hid, generator=g) * 0.1)
    dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
    project = (torch.randn(oup, hid, 1, 1, generator=g) / np.sqrt(hid), torch.randn(oup, generator=g) * 0.1)
    xn = _nhwc(x).to(device)
    y = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res)
    ref = _ref_ir(xn.cpu(), expand, dw, project, s, res)
    _check(_nchw(y.cpu()), ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("B,HW,live", [(3, 7, None), (5, 7, 3), (2, 8, None)])
def test_head_pool_matches_torch(device, B, HW, live):
    """Fused head 1x1 conv (320 -> 1280) + ReLU6 + global average pool vs fp32 torch; crops past the
    device-side live count are not written."""
    g = torch.Generator().manual_seed(B * 10 + HW)
    x = (torch.rand(B, 320, HW, HW, generator=g) * 2).to(torch.bfloat16)
    w = torch.randn(1280, 320, 1, 1, generator=g) / np.sqrt(320)
    b = torch.randn(1280, generator=g) * 0.5
    xn = _nhwc(x).to(device)
    bdev = None if live is None else torch.tensor([live], dtype=torch.int32, device=device)
    y = AF.head_pool_nhwc(xn, w, b, "relu6", bdev=bdev)
    ref = F.relu6(F.conv2d(x.float(), _bf(w), b.float())).mean(dim=(2, 3))
    n = B if live is None else live
    _check(y[:n].float().cpu(), ref[:n], rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,live,f32", [(37, None, True), (20, 9, True), (16, None, False)])
def test_fc_splitk_matches_torch(device, B, live, f32):
    """Classifier FC (1x1 conv on a 1x1 map, 1280 -> 1000) on the split-K kernel vs fp32 torch."""
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 1280, 1, 1, generator=g).to(torch.bfloat16)
    w = torch.randn(1000, 1280, 1, 1, generator=g) / np.sqrt(1280)
    b = torch.randn(1000, generator=g)
    bdev = None if live is None else torch.tensor([live], dtype=torch.int32, device=device)
    y = AF.conv2d_nhwc(_nhwc(x).to(device), w, b, f32out=f32, bdev=bdev)
    ref = F.conv2d(x.float(), _bf(w), b.float())
    n = B if live is None else live
    _check(_nchw(y.cpu()).float()[:n], ref[:n], rtol=1e-2, atol=1e-2)


def test_ir_block_live_batch(device):
    """Crops past the device-side live count are not written."""
    g = torch.Generator().manual_seed(5)
    x = torch.rand(4, 28, 28, 32, generator=g).to(torch.bfloat16).to(device)
    expand = (torch.randn(192, 32, 1, 1, generator=g) / 6, torch.zeros(192))
    dw = (torch.randn(192, 1, 3, 3, generator=g) / 3, torch.zeros(192))
    project = (torch.randn(64, 192, 1, 1, generator=g) / 14, torch.zeros(64))
    bdev = torch.tensor([2], dtype=torch.int32, device=device)
    y = AF.ir_block_nhwc(x, expand, dw, project, stride=2, bdev=bdev)
    full = AF.ir_block_nhwc(x, expand, dw, project, stride=2)
    assert torch.equal(y[:2].cpu(), full[:2].cpu())


@pytest.mark.parametrize(
    "B,H,Cin,Cout",
    [(2, 40, 64, 64), (2, 40, 128, 64), (1, 20, 80, 80), (2, 14, 64, 384), (2, 14, 96, 576), (2, 7, 160, 960),
     (2, 20, 256, 256), (3, 20, 128, 128), (2, 33, 16, 16), (2, 30, 32, 32), (1, 14, 384, 96)],
)
def test_pointwise_fast_path(device, B, H, Cin, Cout):
    """1x1 fast path (conv_pw.hip) vs torch, with residual; and identical to the generic kernel."""
    C = native()
    g = torch.Generator().manual_seed(Cin * 7 + Cout)
    x = torch.randn(B, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) / np.sqrt(Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    xn = _nhwc(x).to(torch.bfloat16).to(device)
    res = torch.randn(B, H, H, Cout, generator=g).to(torch.bfloat16).to(device)
    y = AF.conv2d_nhwc(xn, w, b, act="silu", res=res)
    ref = _ref_conv(xn.cpu(), w, b, 1, 0, "silu", res=res.cpu())
    _check(_nchw(y.cpu()), ref)
    C.set_conv_pw(False)
    try:
        y2 = AF.conv2d_nhwc(xn, w, b, act="silu", res=res)
    finally:
        C.set_conv_pw(True)
    assert (y.float() - y2.float()).abs().max().item() <= 0.0625


def test_pointwise_slices_and_upsample(device):
    g = torch.Generator().manual_seed(17)
    B, H, Cbuf, Cin, Cout = 2, 20, 384, 256, 128
    buf = torch.randn(B, H, H, Cbuf, generator=g).to(torch.bfloat16).to(device)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) / np.sqrt(Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    out = torch.zeros(B, H, H, 256, dtype=torch.bfloat16, device=device)
    up = torch.zeros(B, 2 * H, 2 * H, 192, dtype=torch.bfloat16, device=device)
    AF.conv2d_nhwc(buf, w, b, act="silu", x_coff=64, cin=Cin, out=out, out_coff=128, out2=up, out2_coff=64)
    torch.cuda.synchronize()
    ref = _ref_conv(buf.cpu()[..., 64:64 + Cin], w, b, 1, 0, "silu")
    _check(_nchw(out.cpu()[..., 128:]), ref)
    assert out.cpu()[..., :128].abs().sum() == 0
    upref = F.interpolate(_nchw(out.cpu()[..., 128:]), scale_factor=2, mode="nearest")
    assert torch.equal(_nchw(up.cpu()[..., 64:]), upref)
    assert up.cpu()[..., :64].abs().sum() == 0


@pytest.mark.parametrize("H,Cin,Cout,s", [(40, 64, 64, 1), (80, 64, 144, 1), (20, 256, 144, 1), (40, 128, 256, 2),
                                          (27, 96, 80, 2), (13, 32, 48, 1)])
def test_conv3x3_v3_matches_v2(device, H, Cin, Cout, s):
    """v3 halo-tile kernel == v2 tile kernel (same math, different staging) and close to torch."""
    C = native()
    g = torch.Generator().manual_seed(H + Cin + Cout)
    x = torch.randn(2, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    b = torch.randn(Cout, generator=g) * 0.1
    xn = _nhwc(x).to(torch.bfloat16).to(device)
    y3 = AF.conv2d_nhwc(xn, w, b, stride=s, act="silu")
    C.set_conv_v3(False)
    try:
        y2 = AF.conv2d_nhwc(xn, w, b, stride=s, act="silu")
    finally:
        C.set_conv_v3(True)
    assert (y3.float() - y2.float()).abs().max().item() <= 0.0625
    _check(_nchw(y3.cpu()), _ref_conv(xn.cpu(), w, b, s, 1, "silu"))


def test_executor_autotune_choices(device, tmp_path, monkeypatch):
    """Autotuned conv kernel choices are persisted per (program, bucket) and a table-driven capture runs
    exactly the same kernels: identical choices and bitwise-identical results (engine/tuning.py)."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    yolo, mnet = make_yolo(0, cls_shift=-20.0), make_mobilenet(1)
    imgs = synthetic_images(4, 77)
    monkeypatch.setenv("ARENA_TUNING_FILE", str(tmp_path / "tuning.json"))
    monkeypatch.setenv("ARENA_TUNING", "retune")
    pipe = GpuPipeline(yolo, mnet, device=0, buckets=[4], dtype="bf16")
    assert pipe.tuning_source == "tuned"
    choices = pipe.ex.conv_choices(4)
    # ~50 conv ops remain once the C3 / inverted-residual / stem / head fusions have absorbed the rest
    assert set(c for c in choices if c) <= {1, 2, 3} and sum(1 for c in choices if c) >= 45
    tuned = pipe.infer(imgs)
    monkeypatch.setenv("ARENA_TUNING", "table")
    again = GpuPipeline(yolo, mnet, device=0, buckets=[4], dtype="bf16")
    assert again.tuning_source == "table" and again.ex.conv_choices(4) == choices
    table = again.infer(imgs)
    for a, b in zip(tuned, table):
        assert len(a) == len(b)
        ka, kb = np.lexsort(a.boxes.T), np.lexsort(b.boxes.T)
        np.testing.assert_array_equal(a.boxes[ka], b.boxes[kb])
        np.testing.assert_array_equal(a.topk_logit[ka], b.topk_logit[kb])
    monkeypatch.setenv("ARENA_TUNING", "off")
    plain = GpuPipeline(yolo, mnet, device=0, buckets=[4], dtype="bf16").infer(imgs)
    for a, b in zip(tuned, plain):
        assert abs(len(a) - len(b)) <= 1


@pytest.mark.parametrize("H,s,Cin,Cout", [(64, 1, 16, 32), (64, 2, 16, 32), (37, 1, 16, 32), (40, 1, 80, 80),
                                          (21, 2, 80, 80), (20, 1, 48, 64)])
def test_conv3x3_v3_cin16(device, H, s, Cin, Cout):
    """Cin % 32 == 16 (s2d stems, first C3, the 80-class detect branch) through the v3 halo-tile kernel:
    the last 32-channel slab is half empty."""
    C = native()
    g = torch.Generator().manual_seed(H * 3 + s + Cin)
    x = torch.randn(2, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    b = torch.randn(Cout, generator=g) * 0.1
    xn = _nhwc(x).to(torch.bfloat16).to(device)
    old = C.get_conv_impl()
    C.set_conv_impl(2)
    try:
        C.set_conv_pw(False)
        y = AF.conv2d_nhwc(xn, w, b, stride=s, act="silu")
    finally:
        C.set_conv_pw(True)
        C.set_conv_impl(old)
    _check(_nchw(y.cpu()), _ref_conv(xn.cpu(), w, b, s, 1, "silu"))


@pytest.mark.parametrize("H,inp,hid,oup,res,s", [(112, 32, 32, 16, False, 1), (56, 24, 144, 24, True, 1),
                                                 (28, 32, 192, 32, True, 1), (14, 64, 384, 64, True, 1),
                                                 (20, 24, 144, 24, True, 1), (112, 16, 96, 24, False, 2),
                                                 (56, 24, 144, 32, False, 2)])
def test_ir_wave_matches_block_kernel(device, H, inp, hid, oup, res, s):
    """Wave-per-tile IR kernel (stride 1: 8x8 / 7x7 tiles, stride 2: 4x4) == block-cooperative kernel."""
    C = native()
    g = torch.Generator().manual_seed(H + hid)
    x = (torch.rand(2, inp, H, H, generator=g) * 2).to(torch.bfloat16)
    expand = None if hid == inp else (torch.randn(hid, inp, 1, 1, generator=g) / np.sqrt(inp),
                                      torch.randn(hid, generator=g) * 0.1)
    dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
    project = (torch.randn(oup, hid, 1, 1, generator=g) / np.sqrt(hid), torch.randn(oup, generator=g) * 0.1)
    xn = _nhwc(x).to(device)
    yw = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res)
    C.set_ir_wave(False)
    try:
        yb = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res)
    finally:
        C.set_ir_wave(True)
    assert (yw.float() - yb.float()).abs().max().item() <= 0.07


@pytest.mark.gpu
@pytest.mark.parametrize("B,inp,hid,oup,res", [(3, 64, 384, 64, True), (2, 64, 384, 96, False),
                                                 (3, 96, 576, 96, True)])
def test_ir_block_whole_crop_14(device, B, inp, hid, oup, res):
    """Stride-1 14x14 blocks as one whole-crop tile per workgroup (ARENA_IR_T14) == torch fp32 reference."""
    C = native()
    g = torch.Generator().manual_seed(hid + oup)
    x = (torch.rand(B, inp, 14, 14, generator=g) * 2).to(torch.bfloat16)
    expand = (torch.randn(hid, inp, 1, 1, generator=g) / np.sqrt(inp), torch.randn(hid, generator=g) * 0.1)
    dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
    project = (torch.randn(oup, hid, 1, 1, generator=g) / np.sqrt(hid), torch.randn(oup, generator=g) * 0.1)
    xn = _nhwc(x).to(device)
    C.set_ir_t14(True)
    try:
        y = AF.ir_block_nhwc(xn, expand, dw, project, stride=1, res=res)
    finally:
        C.set_ir_t14(False)
    ref = _ref_ir(xn.cpu(), expand, dw, project, 1, res)
    _check(_nchw(y.cpu()), ref, rtol=3e-2, atol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("H,inp,hid,oup,s,res", [(14, 96, 576, 160, 2, False), (7, 160, 960, 160, 1, True),
                                                 (7, 160, 960, 160, 1, False), (7, 160, 960, 320, 1, False)])
def test_ir_crop_matches_tile_kernel_and_torch(device, H, inp, hid, oup, s, res, split):
    """Whole-crop IR kernel (waves split the hidden channels, ir_crop.hip; ``split`` workgroups per crop
    split its output rows) == torch fp32 reference and the 7x7-tile kernel; crops past the device-side
    live count are not written."""
    C = native()
    C.set_ir_crop_split(split)
    g = torch.Generator().manual_seed(H * 7 + hid)
    x = (torch.rand(5, inp, H, H, generator=g) * 2).to(torch.bfloat16)
    expand = (torch.randn(hid, inp, 1, 1, generator=g) / np.sqrt(inp), torch.randn(hid, generator=g) * 0.1)
    dw = (torch.randn(hid, 1, 3, 3, generator=g) / 3, torch.randn(hid, generator=g) * 0.1)
    project = (torch.randn(oup, hid, 1, 1, generator=g) / np.sqrt(hid), torch.randn(oup, generator=g) * 0.1)
    xn = _nhwc(x).to(device)
    y = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res)
    _check(_nchw(y.cpu()), _ref_ir(xn.cpu(), expand, dw, project, s, res), rtol=3e-2, atol=3e-2)
    C.set_ir_crop(False)
    try:
        yt = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res)
    finally:
        C.set_ir_crop(True)
    assert (y.float() - yt.float()).abs().max().item() <= 0.07
    bdev = torch.tensor([3], dtype=torch.int32, device=device)
    yl = AF.ir_block_nhwc(xn, expand, dw, project, stride=s, res=res, bdev=bdev)
    C.set_ir_crop_split(2)
    assert torch.equal(yl[:3].cpu(), y[:3].cpu())
