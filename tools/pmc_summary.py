#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per-kernel average duration (kernel
trace) and per-kernel average counter values (PMC passes).

    python tools/pmc_summary.py <rocprof_dir> [<rocprof_dir> ...] [--kernel SUBSTR]
Prints JSON: {kernel: {"calls", "avg_ns", counters...}}."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    res = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            with open(f, newline="") as fh:
                rows = list(csv.DictReader(fh))
            if not rows:
                continue
            keys = rows[0].keys()
            if "Counter_Name" in keys:
                for r in rows:
                    k = r.get("Kernel_Name", "")
                    if a.kernel in k:
                        res[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            elif "Start_Timestamp" in keys and "Kernel_Name" in keys:
                for r in rows:
                    k = r["Kernel_Name"]
                    if a.kernel in k:
                        res[k]["duration_ns"].append(
                            float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    out = {}
    for k, cs in res.items():
        out[k] = {c: {"n": len(v), "mean": sum(v) / len(v)} for c, v in cs.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
