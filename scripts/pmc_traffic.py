#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE counter_collection.csv files of two
separate ``rocprofv3 --pmc`` runs (one pass each: FETCH_SIZE takes 3 of the 4
TCC slots, WRITE_SIZE 2) and prints JSON {kernel: {...}} with the per-launch
averages.  Correction (MI355X_MICROARCH.md, HBM): on gfx950 FETCH_SIZE counts
64 B per 128-B request of a wide streaming read, so fetched bytes are taken as
2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Both counters are in KiB.

Usage: python scripts/pmc_traffic.py <fetch_csv> <write_csv> <workload key> [tag]
(workload key as bench.py names it: <workload>_b<pairs>_<dtype>, e.g. sintel_b1_f32)
"""
import collections
import csv
import json
import re
import sys


def per_launch(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name).strip()
        vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    workload = sys.argv[3]
    tag = sys.argv[4] if len(sys.argv) > 4 else ""
    out = {}
    for k in sorted(set(fetch) & set(write)):
        f, w = fetch[k] * 1024, write[k] * 1024
        out[k] = {"fetch_size_bytes": f, "write_size_bytes": w,
                  "traffic_bytes": 2 * f + w, "correction": "2 x FETCH_SIZE + WRITE_SIZE",
                  "source": tag}
    print(json.dumps({"workload": workload, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
