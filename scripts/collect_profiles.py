#!/usr/bin/env python3
"""Copy a round's GPU profile outputs from gpurun_out/<round>/ into profiles/<round>/.

Per config directory: the bench line (bench.json), the bench line of the run under
rocprofv3 (bench_under_rocprof.json), rocprofv3 --stats kernel summary
(kernel_stats.csv), the kernel-trace step timeline (trace_gaps.json), and the
FETCH_SIZE / WRITE_SIZE traffic summary (profiles/<round>/traffic_<config>.json,
read by bench.py).  Also the GPU test log and smoke output when present.
Usage: python scripts/collect_profiles.py r03
"""
from __future__ import annotations

import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def main(tag: str) -> None:
    src, dst = REPO / "gpurun_out" / tag, REPO / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    for d in sorted(p for p in src.iterdir() if p.is_dir()):
        if not (d / "kernel_stats.csv").exists():
            continue
        out = dst / d.name
        out.mkdir(exist_ok=True)
        lines = [ln for ln in (d / "bench.log").read_text().splitlines() if ln.startswith("{")]
        (out / "bench.json").write_text(json.dumps(json.loads(lines[-1]), indent=1) + "\n")
        for f in ("bench_under_rocprof.json", "kernel_stats.csv", "trace_gaps.json",
                  "pmc_FETCH_SIZE.csv", "pmc_WRITE_SIZE.csv"):
            if (d / f).exists():
                shutil.copy(d / f, out / f)
        if (d / "traffic.json").exists():
            shutil.copy(d / "traffic.json", dst / f"traffic_{d.name}.json")
        print("collected", d.name)
    for f, name in (("pytest_gpu.log", "pytest_gpu_final.log"), ("smoke.log", "smoke_final.log")):
        if (src / f).exists():
            shutil.copy(src / f, dst / name)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r03")
