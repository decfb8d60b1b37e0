#!/usr/bin/env python3
"""Map a rocprofv3 kernel trace of the executor back to program ops.

The executor's hipGraph replays the program's ops in order, one kernel per
op, so the k-th arena kernel of each replay is op k.  This tool takes the last
``--replays`` complete replays from ``*_kernel_trace.csv``, averages each op's
duration and prints a per-op table (op index, kind, layer shape, kernel
variant, VGPRs, grid, mean us, share) plus per-kind totals.

    python tools/analyze_trace.py gpurun_out/prof/bench_kernel_trace.csv --bucket 32
"""
from __future__ import annotations

import argparse
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

KIND = {1: "conv", 2: "dwconv", 3: "sppf", 4: "letterbox", 5: "zero", 6: "decode", 7: "nms", 8: "cropplan",
        9: "cropgather", 10: "avgpool", 11: "topk", 12: "tensorin", 13: "yoloraw", 14: "irblock", 15: "stemfused", 16: "c3fused",
        17: "headpool", 18: "stamp"}
FIRST_KERNEL = {4: "letterbox", 12: "tensor_in", 15: "stem_fused", 18: "stamp_kernel"}


def describe(rec) -> str:
    t = int(rec[0])
    if t == 1:
        return (f"{int(rec[4])}x{int(rec[5])}x{int(rec[6])}->{int(rec[13])}x{int(rec[14])}x{int(rec[15])} "
                f"k{int(rec[17])} s{int(rec[19])}{' res' if rec[22] != -1 else ''}{' up2' if rec[25] != -1 else ''}"
                f"{' crops' if rec[30] == 1 else ''}{f' +pw1x1->{int(rec[34])}' if rec[34] > 0 else ''}")
    if t == 2:
        return f"dw {int(rec[4])}x{int(rec[5])}x{int(rec[6])} s{int(rec[14])}"
    if t == 16:
        return (f"c3 {int(rec[4])}x{int(rec[5])}x{int(rec[6])} c_={int(rec[7])} n={int(rec[8])}"
                f"{' res' if rec[9] else ''}")
    if t == 15:
        d = f"{'letterbox' if rec[1] == 0 else 'crop gather'} + stem k{int(rec[19])} -> {int(rec[9])}"
        return d + (f" + k3 s2 -> {int(rec[24])}" if int(rec[20]) else "") + \
            (f" + ir t1 -> {int(rec[31])}" if int(rec[26]) else "")
    if t == 14 and int(rec[31]):
        return f"crop gather + stem -> ir {int(rec[4])}x{int(rec[5])}x{int(rec[6])} -> {int(rec[9])} (t1)"
    if t == 14:
        return (f"ir {int(rec[4])}x{int(rec[5])}x{int(rec[6])}->{int(rec[23])}x{int(rec[24])}x{int(rec[9])} "
                f"hid{int(rec[8])} s{int(rec[11])}{' res' if rec[13] else ''}")
    return ""


def first_kernel(op0) -> str:
    """Name fragment of the kernel that starts one replay of the program (its first op)."""
    first = FIRST_KERNEL.get(int(op0[0]), "letterbox")
    if int(op0[0]) == 15:  # detector stem: single-stage kernel or letterbox+stem+conv (stem2_kernel)
        first = "stem2_kernel" if int(op0[20]) else "stem_fused_kernel<0"
    if int(op0[0]) == 1 and int(op0[1]) == -12:  # fp32 stem conv sampling the letterboxed images (BUF_POOL)
        first = "conv_x3_h16_kernel<1, true>"
    return first


def merge_split_k(q: list[dict]) -> list[dict]:
    """One queue's dispatches in start order, with each split-K conv's second kernel (gemm_x3.hip, impl 171+: the
    partial GEMM, then x3g_sk_reduce_kernel) folded into its op: the reduce's time is added to the GEMM row
    (``_extra_ns``), so one row stays one program op."""
    merged: list[dict] = []
    for r in q:
        if "x3g_sk_reduce_kernel" in r["Kernel_Name"] and merged:
            prev = dict(merged[-1])
            prev["_extra_ns"] = prev.get("_extra_ns", 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            prev["Kernel_Name"] = prev["Kernel_Name"].split("(")[0] + " + sk_reduce("
            merged[-1] = prev
        else:
            merged.append(r)
    return merged


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--replays", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="write the table as markdown")
    ap.add_argument("--dtype", default="bf16", help="program precision the trace was taken with")
    a = ap.parse_args(argv)

    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models

    prog = plan_pipeline(*default_models(a.seed), conf_thr=0.5, iou_thr=0.45, dtype=a.dtype)
    n_ops = prog.ops.shape[0]
    rows = [r for r in csv.DictReader(open(a.trace)) if "arena::" in r["Kernel_Name"]]
    # the executor runs each staging slot on its own stream: slice replays per hardware queue so that
    # kernels of concurrently running graphs are not interleaved
    qkey = next((k for k in ("Queue_Id", "Stream_Id") if rows and k in rows[0]), None)
    by_q = defaultdict(list)
    for r in rows:
        by_q[r[qkey] if qkey else 0].append(r)
    first = first_kernel(prog.ops[0])
    replays = []
    for qk in list(by_q):
        by_q[qk] = merge_split_k(sorted(by_q[qk], key=lambda r: int(r["Start_Timestamp"])))
    for q in by_q.values():
        starts = [i for i, r in enumerate(q) if first in r["Kernel_Name"]]
        replays += [q[s:s + n_ops] for s in starts if s + n_ops <= len(q)]
    replays = [rp for rp in replays if len(rp) == n_ops]
    replays.sort(key=lambda rp: int(rp[0]["Start_Timestamp"]))
    # keep replays whose kernel sequence matches the program's final one (drops slices that straddle
    # autotuning / overflow passes), then use per-op medians
    if replays:
        ref = [r["Kernel_Name"] for r in replays[-1]]
        replays = [rp for rp in replays if [r["Kernel_Name"] for r in rp] == ref]
    replays = replays[-a.replays:]
    if not replays:
        print("no complete replay found", file=sys.stderr)
        return 1
    dur = defaultdict(list)
    for rp in replays:
        for k, r in enumerate(rp):
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) + r.get("_extra_ns", 0)) / 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in dur.items()}
    total = sum(med.values())
    lines = ["| op | kind | shape | kernel | vgpr | grid | mean us | share |", "|---|---|---|---|---|---|---|---|"]
    per_kind = defaultdict(float)
    for k in range(n_ops):
        r = replays[-1][k]
        us = med[k]
        kind = KIND.get(int(prog.ops[k][0]), "?")
        per_kind[kind] += us
        name = r["Kernel_Name"].replace("void arena::", "").replace("arena::", "").split("(")[0]
        grid = f"{int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))}x{r['Grid_Size_Y']}"
        lines.append(f"| {k} | {kind} | {describe(prog.ops[k])} | {name} | {r['VGPR_Count']}+{r['Accum_VGPR_Count']} "
                     f"| {grid} | {us:.1f} | {100 * us / total:.1f}% |")
    lines.append("")
    lines.append(f"replays: {len(replays)} (per-op medians); device time per replay: {total:.1f} us")
    lines.append("")
    lines.append("| kind | us per replay | share |")
    lines.append("|---|---|---|")
    for kind, us in sorted(per_kind.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {kind} | {us:.1f} | {100 * us / total:.1f}% |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
