#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel execution intervals over the traced span
(or over the last ``--window-ms`` of it), plus the number of kernels in flight on average.  Shows whether a
pipelined run is kernel-bound (busy ~100 %) or leaves the device idle between launches.

    python tools/busy_fraction.py gpurun_out/x/..._kernel_trace.csv [--window-ms 500]
"""
from __future__ import annotations

import argparse
import csv
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=0.0, help="only the last N ms of the trace")
    a = ap.parse_args(argv)
    iv = []
    for r in csv.DictReader(open(a.trace)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not iv:
        print("no kernels")
        return 1
    iv.sort()
    t_end = max(e for _, e in iv)
    t0 = iv[0][0] if a.window_ms <= 0 else t_end - int(a.window_ms * 1e6)
    iv = [(max(s, t0), e) for s, e in iv if e > t0]
    busy, cur_s, cur_e, work = 0, None, None, 0
    for s, e in iv:
        work += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - t0
    print(f"span {span / 1e6:.1f} ms, busy {100.0 * busy / span:.1f} %, mean kernels in flight {work / max(busy, 1):.2f}, "
          f"kernels {len(iv)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
