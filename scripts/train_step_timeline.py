#!/usr/bin/env python3
"""Timeline of one eager training step from a rocprofv3 kernel trace (profiles
only): run `rocprofv3 --kernel-trace -- python scripts/time_backward.py
--no-breakdown`, then pass the kernel_trace.csv.  Steps are split at the build's
split pass (split_pairs_kernel); the last complete step is printed kernel by
kernel (start offset, duration, idle before it), with totals: kernel time, idle
time and span, so host-bound stretches show as idle.
Usage: python scripts/train_step_timeline.py <kernel_trace.csv>
"""
from __future__ import annotations

import csv
import json
import re
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    if n.startswith(("at::", "rocblas")):
        return re.sub(r"\(.*", "", n)[:90]   # torch / rocBLAS: the functor names the op
    return re.sub(r"[(<].*", "", n)          # this package's kernels: the name alone


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "split_pairs_kernel" in r[2]]
    if len(starts) < 3:
        print(json.dumps({"error": "fewer than 3 steps in the trace"}))
        return
    a, b = starts[-3], starts[-2]   # the second-to-last complete step
    step = rows[a:b]
    t0 = step[0][0]
    prev_end = None
    out, busy, idle = [], 0, 0
    for s, e, n in step:
        gap = 0 if prev_end is None else max(s - prev_end, 0)
        idle += gap
        busy += e - s
        out.append({"t_us": round((s - t0) / 1e3, 2), "dur_us": round((e - s) / 1e3, 2),
                    "idle_before_us": round(gap / 1e3, 2), "kernel": short(n)})
        prev_end = e if prev_end is None else max(prev_end, e)
    for o in out:
        print(json.dumps(o))
    print(json.dumps({"kernels": len(step), "kernel_us": round(busy / 1e3, 1),
                      "idle_us": round(idle / 1e3, 1),
                      "span_us": round((step[-1][1] - t0) / 1e3, 1)}))


if __name__ == "__main__":
    main()
