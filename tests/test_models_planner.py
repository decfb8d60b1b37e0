"""Model oracles, BN folding, stem rewrites and the executor program planner (CPU)."""
from __future__ import annotations

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from inference_arena_amd.engine.planner import (
    CROPS,
    IMAGES,
    OP_CONV,
    OP_FIELDS,
    ProgramBuilder,
    View,
    layout,
    pack_conv_weight,
)
from inference_arena_amd.engine.plans import plan_pipeline, s2d_stem_3x3, s2d_stem_6x6
from inference_arena_amd.models.common import ConvBNAct, fold, init_random_
from inference_arena_amd.models.mobilenetv2 import MobileNetV2
from inference_arena_amd.models.yolov5nu import YOLOv5nu


def test_yolo_output_contract():
    m = init_random_(YOLOv5nu(), 0).eval()
    with torch.no_grad():
        y = m(torch.rand(1, 3, 320, 320))
    assert y.shape == (1, 84, 2100)  # (40^2 + 20^2 + 10^2) anchors at 320
    assert (y[:, 4:] >= 0).all() and (y[:, 4:] <= 1).all()
    n_conv = sum(isinstance(x, torch.nn.Conv2d) for x in m.modules())
    assert n_conv == 75


def test_mobilenet_output_contract():
    m = init_random_(MobileNetV2(), 1).eval()
    with torch.no_grad():
        y = m(torch.randn(2, 3, 224, 224))
    assert y.shape == (2, 1000)
    assert sum(isinstance(x, torch.nn.Conv2d) for x in m.modules()) == 52
    macs = 0
    hooks = []

    def hk(mod, i, o):
        nonlocal macs
        macs += o.numel() // o.shape[0] * mod.in_channels // mod.groups * mod.kernel_size[0] * mod.kernel_size[1]

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(hk))
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    macs += 1280 * 1000
    assert 295e6 < macs < 305e6  # 0.30 GMAC


def test_bn_fold_equivalence():
    torch.manual_seed(0)
    blk = init_random_(torch.nn.Sequential(ConvBNAct(8, 16, 3, 2)), 3)[0].eval()
    x = torch.randn(2, 8, 9, 9)
    w, b = fold(blk)
    with torch.no_grad():
        ref = blk(x)
        got = F.silu(F.conv2d(x, w, b, stride=2, padding=1))
    assert torch.allclose(ref, got, atol=1e-5)


def _s2d(img):
    B, C, H, W = img.shape
    s = img.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 3, 5, 1, 2, 4).reshape(B, 12, H // 2, W // 2)
    return torch.cat([s, torch.zeros(B, 4, H // 2, W // 2)], 1)


def test_space_to_depth_stems():
    g = torch.Generator().manual_seed(0)
    img = torch.randn(2, 3, 32, 32, generator=g)
    w6 = torch.randn(8, 3, 6, 6, generator=g)
    ref = F.conv2d(img, w6, stride=2, padding=2)
    got = F.conv2d(_s2d(img), s2d_stem_6x6(w6), stride=1, padding=1)
    assert torch.allclose(ref, got, atol=1e-4)
    w3 = torch.randn(8, 3, 3, 3, generator=g)
    ref3 = F.conv2d(img, w3, stride=2, padding=1)
    got3 = F.conv2d(F.pad(_s2d(img), (1, 0, 1, 0)), s2d_stem_3x3(w3))
    assert torch.allclose(ref3, got3, atol=1e-4)


def test_pack_conv_weight_layout():
    w = torch.arange(2 * 3 * 2 * 2, dtype=torch.float32).reshape(2, 3, 2, 2)
    wb, bb, kpad, cpad = pack_conv_weight(w, torch.ones(2))
    assert kpad == 32 and cpad == 16
    arr = torch.frombuffer(bytearray(wb), dtype=torch.bfloat16).float().reshape(cpad, kpad)
    # k = (kh*KW + kw)*Cin + ci
    assert arr[1, (1 * 2 + 0) * 3 + 2].item() == w[1, 2, 1, 0].item()
    assert arr[2:].abs().sum() == 0 and arr[:, 12:].abs().sum() == 0


@pytest.fixture(scope="module")
def program(models):
    return plan_pipeline(*models, conf_thr=0.5, iou_thr=0.45)


def test_program_shape(program):
    assert program.ops.shape[1] == OP_FIELDS
    convs = int((program.ops[:, 0] == OP_CONV).sum())
    # 75 YOLO convs lowered to 64 (C3 cv1+cv2 and the two detect branches' first convs fused);
    # MobileNet: stem + head + FC convs, the 17 inverted-residual blocks as fused ops
    # (unfused: 35 convs = stem + 16 expand + 17 project + head, plus FC)
    from inference_arena_amd.engine.planner import OP_IRBLOCK

    from inference_arena_amd.engine.planner import OP_STEMFUSED

    irs = int((program.ops[:, 0] == OP_IRBLOCK).sum())
    stems = int((program.ops[:, 0] == OP_STEMFUSED).sum())
    # the two stem convs become stem_fused ops (preprocessing fused in) unless ARENA_FUSE_STEM=0
    assert stems in (0, 2)
    convs += stems
    # the detector stem op may also carry the following 3x3 s2 conv (ARENA_FUSE_STEM2)
    convs += int(((program.ops[:, 0] == OP_STEMFUSED) & (program.ops[:, 20] > 0)).sum())
    # ... or MobileNetV2's first inverted residual (ARENA_FUSE_STEM_IR)
    irs += int(((program.ops[:, 0] == OP_STEMFUSED) & (program.ops[:, 26] > 0)).sum())
    # the Detect head's final 1x1 convs ride in the epilogue of the preceding 3x3s unless ARENA_FUSE_HEAD=0
    pw = int(((program.ops[:, 0] == OP_CONV) & (program.ops[:, 34] > 0)).sum())
    assert pw in (0, 6)
    convs += pw
    # whole C3 blocks at 160x160 / 80x80 (cv1|cv2, NB bottlenecks x 2 convs, cv3) unless ARENA_FUSE_C3=0
    from inference_arena_amd.engine.planner import OP_C3FUSED

    c3 = program.ops[program.ops[:, 0] == OP_C3FUSED]
    assert len(c3) in (0, 1, 3)  # none / auto (160x160 block) / all
    convs += int(sum(2 + 2 * int(r[8]) for r in c3))
    # MobileNet head conv + avgpool as one head_pool op unless ARENA_FUSE_POOL=0
    from inference_arena_amd.engine.planner import OP_AVGPOOL, OP_HEADPOOL

    hp = int((program.ops[:, 0] == OP_HEADPOOL).sum())
    assert hp + int((program.ops[:, 0] == OP_AVGPOOL).sum()) == 1
    convs += hp
    # auto policy: blocks 1-16 fused, block 17 (320 out) as expand/project convs (+ 2); ARENA_IR_CROP=0:
    # blocks 14-17 unfused
    assert (convs, irs) in ((64 + 3, 17), (64 + 36, 0), (64 + 3 + 8, 13), (64 + 3 + 2, 16))
    assert program.cls_ops.shape[0] < program.ops.shape[0]
    assert program.weights.nbytes % 256 == 0


def test_unfused_program_shape(models):
    from inference_arena_amd.engine.plans import plan_mobilenet
    from inference_arena_amd.engine.planner import ProgramBuilder

    for fuse, want in ((False, 36), (True, 3)):
        pb = ProgramBuilder()
        crops = pb.raw("crops", 300 * 32)
        plan_mobilenet(pb, models[1], crops, 224, (0.5,) * 3, (0.25,) * 3, fuse_ir=fuse, fuse_stem=False)
        ops = pb.build().ops[:, 0]
        assert int((ops == OP_CONV).sum()) + int((ops == 17).sum()) == want  # head conv may be a head_pool op


@pytest.mark.parametrize("B", [1, 7, 32])
def test_layout_respects_lifetimes(program, B):
    crops = max(16, 8 * B)
    offs, total = layout(program.buffers, B, crops)
    bufs = [b for b in program.buffers if b.last >= 0]
    for i, a in enumerate(bufs):
        sa = a.per_item * (crops if a.kind == CROPS else B)
        assert offs[a.id] % 256 == 0 and offs[a.id] + sa <= total
        for b in bufs[i + 1:]:
            if a.last < b.first or b.last < a.first:
                continue
            sb = b.per_item * (crops if b.kind == CROPS else B)
            assert offs[a.id] + sa <= offs[b.id] or offs[b.id] + sb <= offs[a.id], (a.name, b.name)
    naive = sum(b.per_item * (crops if b.kind == CROPS else B) for b in bufs)
    assert total < 0.5 * naive


def test_builder_validates_shapes():
    pb = ProgramBuilder()
    a = pb.tensor("a", 8, 8, 16)
    b = pb.tensor("b", 8, 8, 32)
    with pytest.raises(ValueError):
        pb.conv(View(a, 0, 16), View(b, 0, 32), torch.zeros(32, 8, 1, 1), torch.zeros(32))
    with pytest.raises(ValueError):
        pb.tensor("bad", 4, 4, 12)
    pb.conv(View(a, 0, 16), View(b, 0, 32), torch.zeros(32, 16, 3, 3), torch.zeros(32), stride=1)
    prog = pb.build()
    assert prog.ops[0, 13] == 8 and prog.ops[0, 30] == IMAGES


@pytest.mark.parametrize("variant", ["pipeline", "detector", "classifier", "yolo_raw", "mobilenet_raw"])
def test_program_variants_validate(variant):
    """Every program variant (fused pipeline, split services, reference tensor models) passes the
    static bounds check for several buckets, and the raw-output programs size their output region."""
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    y, m = default_models(0)
    prog = {
        "pipeline": lambda: plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45),
        "detector": lambda: plans.plan_detector(y, conf_thr=0.5, iou_thr=0.45),
        "classifier": lambda: plans.plan_classifier(m),
        "yolo_raw": lambda: plans.plan_yolo_raw(y),
        "mobilenet_raw": lambda: plans.plan_mobilenet_raw(m),
    }[variant]()
    for B in (1, 3, 32):
        validate_program(prog, B, max(16, 8 * B), max_det=300, cand_cap=8400)
    if variant == "yolo_raw":
        assert prog.meta["raw_out_bytes"] == 84 * 8400 * 4 and prog.meta["output_shape"] == [84, 8400]
    if variant == "mobilenet_raw":
        assert prog.meta["raw_out_bytes"] == 1000 * 4
    if variant == "classifier":
        assert prog.cls_ops.shape[0] > 0  # overflow passes re-run the classifier part


def test_tuning_table_roundtrip(tmp_path, monkeypatch):
    """Persisted conv kernel choices (engine/tuning.py): keyed by program fingerprint and bucket."""
    import numpy as np

    from inference_arena_amd.engine import tuning
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models

    f = tmp_path / "t.json"
    monkeypatch.setenv("ARENA_TUNING_FILE", str(f))
    p = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype="bf16")
    assert tuning.needs_tuning(p.ops)
    assert tuning.needs_tuning(plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype="fp32").ops)
    assert tuning.lookup(p.ops, 8) is None
    ch = [2 if int(o[0]) == 1 else 0 for o in p.ops]
    assert tuning.store(p.ops, 8, ch)
    assert tuning.lookup(p.ops, 8) == ch and tuning.lookup(p.ops, 4) is None
    other = p.ops.copy()
    other[3, 4] += 1
    assert tuning.fingerprint(other) != tuning.fingerprint(p.ops) and tuning.lookup(other, 8) is None
    monkeypatch.setenv("ARENA_TUNING", "bogus")
    assert tuning.mode() == "table"
    assert np.asarray(tuning.load_table()[f"{tuning.fingerprint(p.ops)}:8"]).shape == (len(p.ops),)


def test_split_bf16x3_is_exact_to_fp32_rounding():
    """Triple-bf16 split of the x3 kernels' weights: h + m + l reproduces fp32 values to fp32 rounding."""
    from inference_arena_amd.engine.planner import split_bf16x3

    g = torch.Generator().manual_seed(3)
    t = torch.randn(64, 96, generator=g) * torch.logspace(-4, 3, 96)
    p = split_bf16x3(t)
    assert p.shape == (64, 3, 96) and p.dtype == torch.bfloat16
    back = p[:, 0].double() + p[:, 1].double() + p[:, 2].double()
    rel = ((back - t.double()).abs() / t.double().abs().clamp_min(1e-30)).max().item()
    assert rel <= 2.0 ** -24, rel


def test_fp32_program_with_whole_map_ir_blocks_validates(monkeypatch):
    """ARENA_IRC_F32=1: the fp32 MobileNetV2 14x14 / 7x7 blocks become fused ops with split-plane weights
    (x3w field), sized 6 bytes per weight by the static validator."""
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.planner import OP_IRBLOCK
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    monkeypatch.setenv("ARENA_IRC_F32", "1")
    y, m = default_models(0)
    prog = plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype="fp32")
    ir = [o for o in prog.ops if int(o[0]) == OP_IRBLOCK]
    assert [int(o[4]) for o in ir] == [112, 112, 56, 56, 28, 28, 28] + [14] * 7 + [7] * 3
    # block 1 (stem-fused, exact fp32) has no split weights; the >= 28x28 blocks take the tiled x3 kernel
    assert [int(o[26]) for o in ir] == [1, 0] + [1] * 15  # block 1: x3 stem kernel; block 2: exact fp32
    for B in (1, 32):
        validate_program(prog, B, 6 * B, max_det=300, cand_cap=8400)


@pytest.mark.parametrize("slices", ["1", "3", "6"])
def test_fp32_hidden_sliced_14x14_chain(monkeypatch, slices):
    """ARENA_IRX_SLICES: the stride-1 14x14 blocks (features 8-13) hand partial sums to each other — block 8
    reads a plain tensor, blocks 9-13 read `slices` parts, blocks 8-12 write them, block 13 writes one tensor for
    the unfused 14 -> 7 block; the buffers are sized for the parts (static validator)."""
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.planner import OP_IRBLOCK
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    monkeypatch.setenv("ARENA_IRX_SLICES", slices)
    y, m = default_models(0)
    prog = plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype="fp32")
    ir = [o for o in prog.ops if int(o[0]) == OP_IRBLOCK and int(o[4]) == 14 and int(o[11]) == 1]
    n = int(slices)
    assert [max(1, int(o[27])) for o in ir] == [1] + [n] * 5
    assert [max(1, int(o[28])) for o in ir] == [n] * 5 + [1]
    bufs = {b.id: b for b in prog.buffers}
    for o in ir:
        assert bufs[int(o[20])].C == int(o[9]) * max(1, int(o[28]))
    for B in (1, 32):
        validate_program(prog, B, 6 * B, max_det=300, cand_cap=8400)


@pytest.mark.parametrize("flag,n", [("1", 1), ("0", 0)])
def test_fp32_program_fuses_the_160_c3_block(monkeypatch, flag, n):
    """ARENA_FUSE_C3_F32: the fp32 program runs the 160x160 C3 block (C1 32, c_ 16, one bottleneck) as one op
    with pre-split weight planes (csrc/kernels/c3_x3.hip); the other C3 blocks stay four-conv."""
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.planner import OP_C3FUSED
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    monkeypatch.setenv("ARENA_FUSE_C3_F32", flag)
    y, m = default_models(0)
    prog = plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype="fp32")
    c3 = [o for o in prog.ops if int(o[0]) == OP_C3FUSED]
    assert len(c3) == n
    if n:
        assert [int(v) for v in c3[0][4:10]] == [160, 160, 32, 16, 1, 1] and int(c3[0][47]) == 1
    for B in (1, 32):
        validate_program(prog, B, 6 * B, max_det=300, cand_cap=8400)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_head_lanes_program(monkeypatch, dtype):
    """ARENA_HEAD_LANES: the Detect head's three levels carry lanes 1-3 (side streams in the executor), every other
    op lane 0; buffers the head touches stay live over the whole head region (no arena sharing between
    branches that now run at the same time); off, every op is lane 0 and the program is unchanged."""
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.planner import OP_LANE_FIELD, layout
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    y, m = default_models(0)
    monkeypatch.setenv("ARENA_HEAD_LANES", "0")
    off = plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype=dtype)
    assert not off.ops[:, OP_LANE_FIELD].any()
    monkeypatch.setenv("ARENA_HEAD_LANES", "1")
    on = plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype=dtype)
    lanes = on.ops[:, OP_LANE_FIELD]
    idx = np.nonzero(lanes)[0]
    assert set(lanes[idx].tolist()) == {1, 2, 3}
    assert list(idx) == list(range(idx[0], idx[-1] + 1))  # one contiguous region
    assert list(lanes[idx]) == sorted(lanes[idx])          # level by level
    np.testing.assert_array_equal(np.delete(on.ops, OP_LANE_FIELD, 1), np.delete(off.ops, OP_LANE_FIELD, 1))
    s, e = int(idx[0]), int(idx[-1]) + 1
    for B in (1, 32):
        validate_program(on, B, 6 * B, max_det=300, cand_cap=8400)
        offs, _ = layout(on.buffers, B, 6 * B)
        live = [b for b in on.buffers if b.last >= 0 and b.last >= s and b.first < e]
        for i, a in enumerate(live):
            sa = a.per_item * (6 * B if a.kind == CROPS else B)
            for b in live[i + 1:]:
                sb = b.per_item * (6 * B if b.kind == CROPS else B)
                assert offs[a.id] + sa <= offs[b.id] or offs[b.id] + sb <= offs[a.id], (a.name, b.name)


def test_tuning_table_concurrent_writers(tmp_path):
    """Several processes storing different entries at once (replicas missing the table together): every entry
    survives and the table is valid JSON throughout (one shared .tmp name tore the file)."""
    import json
    import subprocess
    import sys

    table = tmp_path / "t.json"
    code = ("import numpy as np, sys; from inference_arena_amd.engine import tuning; "
            "ops = np.full((3, 48), int(sys.argv[1]), np.int64); "
            f"[tuning.store(ops, b, [b] * 3, __import__('pathlib').Path({str(table)!r})) for b in range(20)]")
    procs = [subprocess.Popen([sys.executable, "-c", code, str(k)]) for k in range(4)]
    assert all(p.wait(120) == 0 for p in procs)
    t = json.loads(table.read_text())
    assert len(t) == 4 * 20
    assert not list(tmp_path.glob("*.tmp"))


def test_pack_conv_weight_x3_layout():
    """Pre-split x3g / x3h weights: [KH*KW*Cin32/32][Cout_pad][h|m|l][32] bf16, each tap's channels padded to
    Cin32, whose planes sum back to the fp32 weights of pack_conv_weight (tap-major K, zeros in the padding)."""
    import numpy as np
    import torch

    from inference_arena_amd.engine.planner import pack_conv_weight, pack_conv_weight_x3

    g = torch.Generator().manual_seed(3)
    for cout, cin, k in [(64, 32, 3), (80, 80, 1), (20, 16, 1), (960, 160, 1), (48, 80, 3)]:
        w = torch.randn(cout, cin, k, k, generator=g)
        b = torch.randn(cout, generator=g)
        wb, _, kpad, cpad = pack_conv_weight(w, b, "fp32")
        ref = np.frombuffer(wb, dtype=np.float32).reshape(cpad, kpad)[:, :k * k * cin].reshape(cpad, k * k, cin)
        cin32 = (cin + 31) // 32 * 32
        raw = np.frombuffer(pack_conv_weight_x3(w), dtype=np.uint16).reshape(k * k * cin32 // 32, cpad, 3, 32)
        planes = torch.from_numpy(raw.astype(np.int32) << 16).view(torch.float32).double()
        full = planes.sum(dim=2).permute(1, 0, 2).reshape(cpad, k * k, cin32).numpy()
        assert np.array_equal(full[:, :, cin:], np.zeros_like(full[:, :, cin:]))
        np.testing.assert_allclose(full[:, :, :cin], ref, rtol=2 ** -23, atol=0)
        assert (planes[:, :, 0].abs() >= planes[:, :, 1].abs()).all()
