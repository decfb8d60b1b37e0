#!/usr/bin/env python3
"""Per-op hardware-counter table from rocprofv3 --pmc runs of bench.py.

Each ``<dir>/run_counter_collection.csv`` holds one counter set for every
dispatch.  The program's ops are located as in analyze_trace.py (a replay
starts at the letterbox kernel; the k-th arena dispatch of a replay is op k);
values are averaged over the last complete replays and per-op ratios are
derived: VALU and LDS instructions per MFMA, LDS bank-conflict share, waves,
and the MFMA-busy share of the SIMDs (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).

    python tools/analyze_pmc.py gpurun_out/pmc2/*/run_counter_collection.csv --out profiles/r1_pmc_ops.md
"""
from __future__ import annotations

import argparse
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def dispatch_us(counter_csv: Path) -> dict[int, float]:
    """Kernel durations (us) by Dispatch_Id from the same run's kernel trace (``rocprofv3 --pmc ... --kernel-trace``
    writes ``*kernel_trace.csv`` next to ``*counter_collection.csv``); {} when the run had no trace."""
    out: dict[int, float] = {}
    for t in sorted(counter_csv.parent.glob("*kernel_trace.csv")):
        for r in csv.DictReader(open(t)):
            try:
                out[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            except (KeyError, ValueError):
                continue
    return out


def replays(path: Path, n_ops: int, keep: int, first: str = "letterbox"):
    rows = [r for r in csv.DictReader(open(path)) if "arena::" in r["Kernel_Name"]]
    by_dispatch = defaultdict(dict)
    names = {}
    durs = dispatch_us(path)
    for r in rows:
        d = int(r["Dispatch_Id"])
        by_dispatch[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
        if d in durs:
            by_dispatch[d]["_us"] = durs[d]
    order = sorted(by_dispatch)
    starts = [i for i, d in enumerate(order) if first in names[d]]
    out = []
    for s in starts:
        seq = order[s:s + n_ops]
        if len(seq) == n_ops:
            out.append([(names[d], by_dispatch[d]) for d in seq])
    return out[-keep:]


def main(argv=None) -> int:
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models
    from tools.analyze_trace import KIND, describe, first_kernel

    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--replays", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--times", default=None, help="per-op table of analyze_trace.py (mean us) for achieved TB/s")
    a = ap.parse_args(argv)
    times = {}
    if a.times:
        for line in Path(a.times).read_text().splitlines():
            cells = [c.strip() for c in line.strip().strip("|").split("|")]
            if len(cells) >= 7 and cells[0].isdigit():
                try:
                    times[int(cells[0])] = float(cells[6])
                except ValueError:
                    pass
    prog = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype=a.dtype)
    n_ops = prog.ops.shape[0]
    vals = defaultdict(lambda: defaultdict(list))
    kname = {}
    for f in a.csvs:
        for rp in replays(Path(f), n_ops, a.replays, first_kernel(prog.ops[0])):
            for k, (name, cnt) in enumerate(rp):
                kname[k] = name.replace("void arena::", "").split("(")[0]
                for c, v in cnt.items():
                    vals[k][c].append(v)
    counters = sorted({c for k in vals for c in vals[k] if not c.startswith("_")})
    lines = ["| op | kind | shape | kernel | " + " | ".join(counters)
             + " | valu/mfma | lds/mfma | conflict % | mfma busy % | wait % | HBM MB (rd+wr) | us | TB/s |",
             "|" + "---|" * (4 + len(counters) + 8)]
    for k in range(n_ops):
        if k not in vals:
            continue
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        mf = m.get("SQ_INSTS_MFMA", 0.0)
        vr = f"{m['SQ_INSTS_VALU'] / mf:.1f}" if mf and "SQ_INSTS_VALU" in m else "-"
        lr = f"{m['SQ_INSTS_LDS'] / mf:.2f}" if mf and "SQ_INSTS_LDS" in m else "-"
        cf = (f"{100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1f}"
              if m.get("SQ_LDS_IDX_ACTIVE") else "-")
        # MFMA busy share of the SIMDs while the kernel runs: SQ_VALU_MFMA_BUSY_CYCLES is summed over the
        # 1024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs (GRBM/8 reproduces the kernel-trace durations)
        mb = (f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.1f}"
              if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m else "-")
        # share of wave cycles spent waiting (s_waitcnt / barrier / dependency), SQ_WAIT_ANY over SQ_WAVE_CYCLES
        wt = (f"{100 * m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.0f}"
              if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m else "-")
        # FETCH_SIZE / WRITE_SIZE are KiB of L2 <-> memory traffic (the HBM side of the kernel)
        mbytes = (m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) * 1024 / 1e6
        hb = f"{mbytes:.1f}" if ("FETCH_SIZE" in m or "WRITE_SIZE" in m) else "-"
        # duration: this run's kernel trace (the counters' own dispatches) or, failing that, an analyze_trace table
        us = m.get("_us") or times.get(k)
        us = round(us, 1) if us else None
        tbs = f"{mbytes * 1e6 / (us * 1e-6) / 1e12:.2f}" if us and hb != "-" else "-"
        kind = KIND.get(int(prog.ops[k][0]), "?")
        lines.append(f"| {k} | {kind} | {describe(prog.ops[k])} | {kname[k]} | "
                     + " | ".join(f"{m[c]:.3g}" if c in m else "-" for c in counters)
                     + f" | {vr} | {lr} | {cf} | {mb} | {wt} | {hb} | {us if us else '-'} | {tbs} |")
    lines.append("")
    lines.append("FETCH_SIZE / WRITE_SIZE are the L2 <-> memory (fabric) request counters; on gfx950 FETCH_SIZE reports "
                 "half the bytes of wide 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), so TB/s of "
                 "read-dominated kernels is a lower bound; us from the run's kernel trace (--kernel-trace).")
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
