"""tools/analyze_pmc.py attribution: counters map to ops per queue and by kernel name, and a
window whose counted durations disagree with the op table fails the duration check."""
from __future__ import annotations

import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from tools import analyze_pmc as P  # noqa: E402

# a 4-op "program": 3x3 conv, 1x1 conv, 3x3 conv, 1x1 conv (the op-7/8 neighbourhood of the round-5 table)
OPS = [("conv_x3_halo_kernel<2, 8>", 40.0, 7.7e5), ("conv_x3_stream_kernel<2, 1>", 12.0, 1.9e5),
       ("conv_x3_halo_kernel<2, 8>", 40.0, 7.7e5), ("conv_x3_stream_kernel<2, 1>", 12.0, 1.9e5)]
FLOOR_US, MHZ = 20.0, 2000.0


def _write(path: Path, dispatches: list[tuple[int, str, str, float, float]]) -> None:
    """dispatches: (dispatch id, queue, kernel, us traced, mfma count) -> a run_counter_collection.csv"""
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Queue_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
                    "End_Timestamp"])
        t = 1_000_000
        for d, q, name, us, mfma in dispatches:
            dur = us + FLOOR_US
            end = t + int(dur * 1e3)
            full = f"void arena::{name}(arena::ConvParams)" if not name.startswith("__") else name
            w.writerow([d, q, full, "SQ_INSTS_MFMA", mfma, t, end])
            w.writerow([d, q, full, "GRBM_GUI_ACTIVE", dur * MHZ * 8, t, end])
            t = end + 5000


def _replay(start_id: int, q: str, skip: int | None = None):
    out, d = [], start_id
    for k, (name, us, mf) in enumerate(OPS):
        if k == skip:
            continue
        out.append((d, q, name, us, mf))
        d += 2
    return out


def test_norm_name_matches_op_table():
    assert P.norm_name("void arena::conv_x3g_kernel<4, 2, 1, 1, false>(arena::ConvParams)") == \
        "conv_x3g_kernel<4, 2, 1, 1, false>"
    assert P.norm_name("arena::stamp_kernel(unsigned long*)") == "stamp_kernel"


def test_interleaved_queues_and_missing_dispatch_map_by_name(tmp_path):
    # two slots' replays interleave in dispatch order (even ids on queue 1, odd on queue 2); queue 2's second
    # replay lost a dispatch (op 1): position-only slicing would hand op 2's counters to op 1
    rows = _replay(0, "1") + _replay(1, "2") + _replay(20, "1") + _replay(21, "2", skip=1)
    rows.append((40, "1", "__amd_rocclr_fillBufferAligned", 3.0, 0.0))  # a runtime kernel between replays
    rows += _replay(42, "1")
    rows.sort()
    f = tmp_path / "run_counter_collection.csv"
    _write(f, rows)
    by_q = P.load_dispatches(f)
    reps = P.find_replays(by_q, [n for n, _, _ in OPS], keep=10)
    assert len(reps) == 4  # the broken window is not a replay
    for rp in reps:
        assert [d["name"] for d in rp] == [n for n, _, _ in OPS]
        assert [d["counters"]["SQ_INSTS_MFMA"] for d in rp] == [m for _, _, m in OPS]


def test_duration_check_flags_misattributed_counters():
    times = {k: us for k, (_, us, _) in enumerate(OPS)}
    good = {k: {"GRBM_GUI_ACTIVE": [(us + FLOOR_US) * MHZ * 8]} for k, us in times.items()}
    dur = {k: [us + FLOOR_US] for k, us in times.items()}
    bad, us_grbm = P.duration_check(good, dur, times, 0.30)
    assert bad == [] and abs(us_grbm[1] - (12.0 + FLOOR_US)) < 1e-6
    # op 1 (a 12 us 1x1) carrying the counters of the 40 us 3x3 next to it
    wrong = {k: dict(v) for k, v in good.items()}
    wrong[1] = {"GRBM_GUI_ACTIVE": list(good[0]["GRBM_GUI_ACTIVE"])}
    bad, _ = P.duration_check(wrong, dur, times, 0.30)
    assert len(bad) == 1 and bad[0].startswith("op 1:")


def test_split_k_reduce_counts_to_its_op(tmp_path):
    """A split-K conv dispatches the partial GEMM and x3g_sk_reduce_kernel; the op table (analyze_trace) names the op
    "<gemm> + sk_reduce", and the counters of both dispatches belong to it."""
    gemm = "conv_x3g_kernel<2, 2, 1, 1, false, true>"
    rows = [(0, "1", "conv_x3_halo_kernel<2, 8>", 40.0, 7.7e5), (2, "1", gemm, 10.0, 3.0e5),
            (4, "1", "x3g_sk_reduce_kernel", 3.0, 0.0), (6, "1", "conv_x3_stream_kernel<2, 1>", 12.0, 1.9e5)]
    f = tmp_path / "run_counter_collection.csv"
    _write(f, rows)
    by_q = P.load_dispatches(f)
    names = [d["name"] for d in by_q["1"]]
    assert names == ["conv_x3_halo_kernel<2, 8>", gemm + " + sk_reduce", "conv_x3_stream_kernel<2, 1>"]
    sk = by_q["1"][1]
    assert sk["counters"]["SQ_INSTS_MFMA"] == 3.0e5
    assert sk["counters"]["GRBM_GUI_ACTIVE"] == ((10.0 + FLOOR_US) + (3.0 + FLOOR_US)) * MHZ * 8
