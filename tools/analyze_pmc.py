#!/usr/bin/env python3
"""Per-op hardware-counter table from rocprofv3 --pmc runs of the engine, with attribution checks.

Each ``<dir>/run_counter_collection.csv`` holds one counter set for every dispatch of one run.  Ops are mapped
to dispatches the way tools/analyze_trace.py maps a kernel trace, plus two checks that the round-5 table lacked
(1x1 convs carried the counters of the neighbouring 3x3 convs):

* **per queue, by name.**  Dispatches are sliced per ``Queue_Id`` (each staging slot's graph runs on its own
  stream, so replays of concurrent batches interleave in ``Dispatch_Id`` order) and a window of dispatches is a
  replay only when EVERY kernel name equals the name the op table (``--times``, the same program's
  analyze_trace.py table) lists for that op.  Windows that straddle a replay boundary, a missing dispatch or
  another stream's work therefore never map;
* **duration.**  Every set carries ``GRBM_GUI_ACTIVE`` (cycles summed over the 8 XCDs).  Per op,
  GRBM/8 / clock is the counted dispatch's duration under profiling; the clock is fitted on the run's own long
  dispatches (their ``End - Start``) and the per-dispatch profiling floor is the median excess over the op
  table's un-profiled duration.  An op whose counted duration minus the floor differs from its op-table duration
  by more than ``--tol`` (30 %) + 2 us fails the tool (exit 2): its counters describe some other dispatch.

Derived columns: VALU and LDS instructions per MFMA, LDS bank-conflict share, MFMA-busy share of the SIMDs
(SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), wait share (SQ_WAIT_ANY over
SQ_WAVE_CYCLES), HBM bytes and TB/s over the op table's duration.

    python tools/analyze_pmc.py gpurun_out/T/pmc/s*/run_counter_collection.csv --dtype fp32 \\
        --times gpurun_out/T/ops_bs32.md --out profiles/T/ops_pmc.md
"""
from __future__ import annotations

import argparse
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def norm_name(name: str) -> str:
    """Kernel name as the op table prints it: no return type, no ``arena::`` qualifiers, no argument list."""
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("arena::", "")
    depth = 0
    for i, ch in enumerate(n):  # cut the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i].strip()
    return n.strip()


def read_op_table(path: Path) -> tuple[dict[int, float], dict[int, str]]:
    """analyze_trace.py markdown table -> ({op: mean us}, {op: kernel name})."""
    times, names = {}, {}
    for line in Path(path).read_text().splitlines():
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) >= 7 and cells[0].isdigit():
            k = int(cells[0])
            names[k] = cells[3]
            try:
                times[k] = float(cells[6])
            except ValueError:
                pass
    return times, names


def load_dispatches(counter_csv: Path) -> dict[str, list[dict]]:
    """{queue: [dispatch, ...] in dispatch order}; a dispatch = {id, name, start, end, counters{}}."""
    by_id: dict[int, dict] = {}
    for r in csv.DictReader(open(counter_csv)):
        if "arena::" not in r["Kernel_Name"]:  # torch / runtime kernels (fills, copies) are not program ops
            continue
        d = int(r["Dispatch_Id"])
        e = by_id.get(d)
        if e is None:
            e = by_id[d] = {"id": d, "name": norm_name(r["Kernel_Name"]), "queue": r.get("Queue_Id", "0"),
                            "start": int(r.get("Start_Timestamp") or 0), "end": int(r.get("End_Timestamp") or 0),
                            "counters": {}}
        e["counters"][r["Counter_Name"]] = e["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    by_q: dict[str, list[dict]] = defaultdict(list)
    for d in sorted(by_id):
        e = by_id[d]
        q = by_q[e["queue"]]
        if e["name"] == "x3g_sk_reduce_kernel" and q:
            # a split-K conv's second kernel (gemm_x3.hip): its counters and time count to the op, as in the op
            # table (tools/analyze_trace.py merge_split_k names the op "<gemm kernel> + sk_reduce")
            prev = q[-1]
            for k, v in e["counters"].items():
                prev["counters"][k] = prev["counters"].get(k, 0.0) + v
            prev["end"] = max(prev["end"], e["end"])
            if not prev["name"].endswith(" + sk_reduce"):
                prev["name"] += " + sk_reduce"
            continue
        q.append(e)
    return by_q


def find_replays(by_q: dict[str, list[dict]], expected: list[str], keep: int) -> list[list[dict]]:
    """Windows of consecutive same-queue dispatches whose names equal ``expected`` op for op (last ``keep``)."""
    n = len(expected)
    out = []
    for q in by_q.values():
        names = [d["name"] for d in q]
        i = 0
        while i + n <= len(q):
            if names[i] == expected[0] and names[i:i + n] == expected:
                out.append(q[i:i + n])
                i += n
            else:
                i += 1
    out.sort(key=lambda rp: rp[0]["id"])
    return out[-keep:]


def duration_check(vals: dict[int, dict[str, list[float]]], dur_pmc: dict[int, list[float]], times: dict[int, float],
                   tol: float) -> tuple[list[str], dict[int, float]]:
    """GRBM-derived duration of each op's counted dispatches against the op table: (problems, {op: us_grbm})."""
    samples = [(statistics.median(vals[k]["GRBM_GUI_ACTIVE"]) / 8.0, statistics.median(dur_pmc[k]))
               for k in vals if "GRBM_GUI_ACTIVE" in vals[k] and dur_pmc.get(k)]
    long_ = [c / us for c, us in samples if us >= 30.0]
    if not long_:
        return ["no dispatch of >= 30 us to fit the clock on"], {}
    mhz = statistics.median(long_)
    us_grbm = {k: statistics.median(vals[k]["GRBM_GUI_ACTIVE"]) / 8.0 / mhz for k in vals if "GRBM_GUI_ACTIVE" in vals[k]}
    excess = [us_grbm[k] - times[k] for k in us_grbm if k in times]
    if not excess:
        return ["no op-table duration to compare with"], us_grbm
    floor = statistics.median(excess)
    bad = []
    for k in sorted(us_grbm):
        if k not in times or times[k] < 8.0:  # launch-sized ops sit inside the floor's spread
            continue
        got = us_grbm[k] - floor
        if abs(got - times[k]) > tol * times[k] + 2.0:
            bad.append(f"op {k}: counted {got:.1f} us (after the {floor:.1f} us floor) vs {times[k]:.1f} us traced")
    return bad, us_grbm


def main(argv=None) -> int:
    from inference_arena_amd.engine.plans import plan_pipeline
    from inference_arena_amd.models.zoo import default_models
    from tools.analyze_trace import KIND, describe

    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--replays", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--times", required=True,
                    help="per-op table of analyze_trace.py for the same program: kernel names (attribution) and "
                         "un-profiled durations (duration check, TB/s)")
    ap.add_argument("--tol", type=float, default=0.30)
    ap.add_argument("--no-check", action="store_true", help="report duration disagreements without failing")
    a = ap.parse_args(argv)
    times, tnames = read_op_table(Path(a.times))
    prog = plan_pipeline(*default_models(0), conf_thr=0.5, iou_thr=0.45, dtype=a.dtype)
    n_ops = prog.ops.shape[0]
    if sorted(tnames) != list(range(n_ops)):
        print(f"op table lists ops {min(tnames, default=-1)}..{max(tnames, default=-1)}, program has {n_ops}",
              file=sys.stderr)
        return 2
    expected = [tnames[k] for k in range(n_ops)]
    problems = []
    vals: dict[int, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    per_set = []
    for f in a.csvs:
        reps = find_replays(load_dispatches(Path(f)), expected, a.replays)
        if not reps:
            problems.append(f"{f}: no window of dispatches matches the op table's kernel sequence")
            continue
        sv: dict[int, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
        dur: dict[int, list[float]] = defaultdict(list)
        for rp in reps:
            for k, d in enumerate(rp):
                for c, v in d["counters"].items():
                    vals[k][c].append(v)
                    sv[k][c].append(v)
                if d["end"] > d["start"]:
                    dur[k].append((d["end"] - d["start"]) * 1e-3)
        bad, _ = duration_check(sv, dur, times, a.tol)
        per_set.append((f, len(reps), sorted({c for k in sv for c in sv[k]})))
        problems += [f"{f}: {b}" for b in bad]
    counters = sorted({c for k in vals for c in vals[k]})
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
        # MFMA busy share of the SIMDs while the kernel runs: SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1024
        # SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs; both from the same set (the busy counter's own pass)
        mb = (f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.1f}"
              if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m else "-")
        # share of wave cycles parked in s_waitcnt / barriers: SQ_WAIT_ANY over SQ_WAVE_CYCLES (same units)
        wt = (f"{100 * m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.0f}"
              if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m else "-")
        mbytes = (m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) * 1024 / 1e6
        hb = f"{mbytes:.1f}" if ("FETCH_SIZE" in m or "WRITE_SIZE" in m) else "-"
        us = times.get(k)
        tbs = f"{mbytes * 1e6 / (us * 1e-6) / 1e12:.2f}" if us and hb != "-" else "-"
        kind = KIND.get(int(prog.ops[k][0]), "?")
        lines.append(f"| {k} | {kind} | {describe(prog.ops[k])} | {expected[k]} | "
                     + " | ".join(f"{m[c]:.3g}" if c in m else "-" for c in counters)
                     + f" | {vr} | {lr} | {cf} | {mb} | {wt} | {hb} | {us if us else '-'} | {tbs} |")
    lines.append("")
    lines.append("Attribution: per-queue windows whose kernel names equal the op table's, op for op; sets: "
                 + "; ".join(f"{Path(f).parent.name} {n} replays ({', '.join(c)})" for f, n, c in per_set) + ".")
    lines.append(f"Duration check (GRBM_GUI_ACTIVE / 8 / fitted clock, minus the profiling floor, vs the op table; "
                 f"tolerance {int(a.tol * 100)} % + 2 us, ops of >= 8 us): " + ("passed" if not problems else f"{len(problems)} problems"))
    lines += [f"- {p}" for p in problems]
    lines.append("FETCH_SIZE / WRITE_SIZE are the L2 <-> memory (fabric) request counters; on gfx950 FETCH_SIZE reports "
                 "half the bytes of wide 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), so TB/s of "
                 "read-dominated kernels is a lower bound; us = the op table's un-profiled duration.")
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    if problems:
        print("\n".join(problems), file=sys.stderr)
        return 0 if a.no_check else 2
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
