#!/usr/bin/env python3
"""Step timeline from a rocprofv3 kernel trace of bench.py (profiles only).

A step of the bench is one build (or, for the on-the-fly block, its pools /
layout kernels) followed by 12 lookups.  For every step whose build kernels are
followed by exactly 12 lookup kernels and then the next step's build (the back-to-back
replays of the clock warm-up, the warmup steps and the timed steps), this
reports medians of: the build kernels' duration, the lookup kernels' durations,
the step span (build start to next build start), and the idle time of the span
(span minus the kernels' durations: kernel boundaries and graph launches), split
by boundary: inside the build (split pass -> DMA build), build -> first lookup,
between the lookups, and last lookup -> the next step's build (the graph
replay boundary); the build's in-step span and the first lookup's duration.
With several steps per graph (bench.py --steps-per-graph) only every G-th
step_to_step boundary is a graph replay boundary, so the idle times are also
reported as means over the steps (the per-step cost the bench's value sees).

Usage: python scripts/trace_gaps.py <run_kernel_trace.csv> [workload key, e.g. sintel_b1_f32]
"""
from __future__ import annotations

import csv
import json
import sys

import numpy as np


def main(path: str, workload: str | None = None) -> None:
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    prod = ("corr_build", "split_pairs", "pack_bf16", "pool", "transpose")
    # forward lookups: the query-minor kernel (round 6) or the wide one (rounds 1-5)
    is_look = [("corr_lookup_qm_kernel" in n or "corr_lookup_wide_kernel" in n or
                "alt_corr_mfma_kernel" in n) for _, _, n in rows]
    # the ordered on-the-fly lookup's three ordering launches belong to its lookup
    is_aux = [("alt_bin_" in n) for _, _, n in rows]
    is_prep = [any(p in n for p in prod) and not is_look[i] and not is_aux[i]
               for i, (_, _, n) in enumerate(rows)]
    # step starts: a build-side kernel right after a lookup (or first in the trace)
    starts = [i for i in range(len(rows)) if is_prep[i] and (i == 0 or is_look[i - 1])]
    b_us, l_us, x_us, span_us, idle_us = [], [], [], [], []
    bspan_us, l1_us, gaps = [], [], {"in_build": [], "build_to_lookup": [], "between_lookups": [],
                                     "step_to_step": []}
    for a, b in zip(starts, starts[1:]):
        looks = [i for i in range(a, b) if is_look[i]]
        aux = [i for i in range(a, b) if is_aux[i]]
        prep = [i for i in range(a, b) if is_prep[i]]
        if len(looks) != 12 or len(looks) + len(aux) + len(prep) != b - a:
            continue
        b_us.append(sum(rows[i][1] - rows[i][0] for i in prep) / 1e3)
        l_us.extend((rows[i][1] - rows[i][0]) / 1e3 for i in looks)
        l1_us.append((rows[looks[0]][1] - rows[looks[0]][0]) / 1e3)
        x_us.append(sum(rows[i][1] - rows[i][0] for i in aux) / 1e3 / 12)
        span = (rows[b][0] - rows[a][0]) / 1e3
        busy = sum((rows[i][1] - rows[i][0]) for i in range(a, b)) / 1e3
        span_us.append(span)
        idle_us.append(span - busy)
        # the build as the step sees it: first build kernel start to last build kernel end
        bspan_us.append((rows[prep[-1]][1] - rows[prep[0]][0]) / 1e3)
        gap = lambda i: max(rows[i + 1][0] - rows[i][1], 0) / 1e3  # noqa: E731
        gaps["in_build"].append(sum(gap(i) for i in prep[:-1]))
        gaps["build_to_lookup"].append(gap(prep[-1]))
        gaps["between_lookups"].append(sum(gap(i) for i in range(prep[-1] + 1, b - 1)))
        gaps["step_to_step"].append(gap(b - 1))
    if not b_us:
        print(json.dumps({"steps": 0, "note": "no build + 12 lookup steps found"}))
        return
    med = lambda v: round(float(np.median(v)), 2)  # noqa: E731
    mean = lambda v: round(float(np.mean(v)), 2)  # noqa: E731
    print(json.dumps({
        **({"workload": workload} if workload else {}),
        "steps": len(b_us),
        "build_us_median": med(b_us), "lookup_us_median": med(l_us),
        "lookup_order_us_median": med(x_us),
        "step_span_us_median": med(span_us), "idle_us_per_step_median": med(idle_us),
        "build_in_step_us_median": med(bspan_us), "first_lookup_us_median": med(l1_us),
        "idle_us_median_by_boundary": {k: med(v) for k, v in gaps.items()},
        "step_span_us_mean": mean(span_us), "idle_us_per_step_mean": mean(idle_us),
        "idle_us_mean_by_boundary": {k: mean(v) for k, v in gaps.items()},
        "what": "back-to-back steps of the bench's step graph: build + 12 lookups, from the "
                "rocprofv3 kernel trace of the same command (durations are kernel begin-end; "
                "lookup_order_us: the on-the-fly lookup's ordering launches per lookup)",
    }))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
