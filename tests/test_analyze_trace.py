"""tools/analyze_trace.py: a split-K conv is two kernels (the partial GEMM and x3g_sk_reduce_kernel) but one program
op; the op table must count the reduce's time to that op and keep one row per op."""
from __future__ import annotations

import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _tool():
    spec = importlib.util.spec_from_file_location("analyze_trace", ROOT / "tools" / "analyze_trace.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _row(name, t0, t1):
    return {"Kernel_Name": name, "Start_Timestamp": str(t0), "End_Timestamp": str(t1)}


def test_split_k_reduce_is_folded_into_its_op():
    t = _tool()
    q = [_row("void arena::stem_s2_x3_kernel<4, 4>(arena::StemFusedParams)", 0, 10_000),
         _row("void arena::conv_x3g_kernel<2, 2, 1, 1, false, true>(arena::ConvParams)", 12_000, 19_000),
         _row("arena::x3g_sk_reduce_kernel(arena::ConvParams)", 20_000, 23_000),
         _row("arena::nms_kernel(arena::NmsParams)", 25_000, 30_000)]
    m = t.merge_split_k(q)
    assert len(m) == 3
    assert "sk_reduce" in m[1]["Kernel_Name"] and m[1]["_extra_ns"] == 3_000
    assert m[2]["Kernel_Name"].startswith("arena::nms_kernel")
    # a leading reduce (no GEMM before it in this queue slice) stays a row of its own
    assert len(t.merge_split_k(q[2:])) == 2
