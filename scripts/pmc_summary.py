#!/usr/bin/env python3
"""Summarise gpu_pmc.sh passes: per kernel, the average of every counter per
dispatch, plus derived ratios (fractions of SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE).
Usage: python scripts/pmc_summary.py gpurun_out/<tag>"""
import collections
import csv
import json
import re
import sys
from pathlib import Path

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(Path(sys.argv[1]).glob("p*.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")
                   .replace("void ", "")).strip()
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in vals.items():
    a = {c: sum(v) / len(v) for c, v in d.items()}
    wc = a.get("SQ_WAVE_CYCLES")
    der = {}
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if c in a:
                der[c + "/WAVE_CYCLES"] = round(a[c] / wc, 3)
    if "SQ_LDS_BANK_CONFLICT" in a and a.get("SQ_LDS_IDX_ACTIVE"):
        der["LDS_conflict/active"] = round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"], 3)
    if "TCC_HIT_sum" in a and "TCC_MISS_sum" in a:
        der["TCC_hit_rate"] = round(a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"]), 3)
    if "TCP_TCC_READ_REQ_LATENCY_sum" in a and a.get("TCP_TCC_READ_REQ_sum"):
        der["L1_L2_read_latency_cyc"] = round(a["TCP_TCC_READ_REQ_LATENCY_sum"] / a["TCP_TCC_READ_REQ_sum"], 1)
    if "FETCH_SIZE" in a:
        der["fetch_bytes_x2"] = 2 * a["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in a:
        der["write_bytes"] = a["WRITE_SIZE"] * 1024
    out[k] = {"counters": {c: round(v, 1) for c, v in a.items()}, "derived": der,
              "dispatches": max(len(v) for v in d.values())}
print(json.dumps(out, indent=1))
