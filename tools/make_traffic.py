#!/usr/bin/env python3
"""Builds profiles/traffic.json (read by bench.py) from rocprofv3 PMC passes,
following MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from
separate passes (TCC slot limit), are in KiB per dispatch, and FETCH_SIZE is
corrected by the factor measured on a known-byte run of the same access
pattern (tools/pmc_calibrate.py: every B row gathered exactly once).

    python tools/make_traffic.py gpurun_out/prof [--out profiles/traffic.json]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def summary(d, kernel):
    out = subprocess.run([sys.executable, os.path.join(HERE, "pmc_summary.py"), d, "--kernel",
                          kernel], capture_output=True, text=True, check=True).stdout
    res = json.loads(out)
    assert len(res) == 1, f"{d}: expected one kernel matching {kernel}, got {list(res)}"
    return next(iter(res.values()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("--kernel", default="csr_mergepath_kernel")
    ap.add_argument("--calib-reads", type=float, required=True)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--nnz", type=int, default=61859140)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(HERE), "profiles",
                                                  "traffic.json"))
    a = ap.parse_args()
    p = a.prof
    fetch = summary(os.path.join(p, "fetch"), a.kernel)["FETCH_SIZE"]["mean"] * 1024
    write = summary(os.path.join(p, "write"), a.kernel)["WRITE_SIZE"]["mean"] * 1024
    cfetch = summary(os.path.join(p, "cfetch"), a.kernel)["FETCH_SIZE"]["mean"] * 1024
    factor = a.calib_reads / cfetch
    hbm = fetch * factor + write
    rec = {"K": a.K, "nnz": a.nnz, "kernel": a.kernel,
           "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
           "fetch_correction": round(factor, 4),
           "calibration": {"known_read_bytes": a.calib_reads, "fetch_size_bytes": round(cfetch)},
           "hbm_bytes_per_launch": round(hbm)}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
