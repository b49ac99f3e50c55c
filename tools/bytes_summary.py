#!/usr/bin/env python3
"""Counter bytes of each workload's dominant kernel from tools/pmc_bytes.sh's
passes: FETCH_SIZE (KiB per dispatch) x the calibration factor + WRITE_SIZE,
per launch, against the kernel-trace mean duration of the same kernel, and
beside the bench line's own byte model (roofline.bytes_per_launch). Each
record carries the bench line's roofline.traffic_key, the exact shape
bench.py will use it for.

    python tools/bytes_summary.py gpurun_out/pmcb WORKLOAD [WORKLOAD ...]
Prints one JSON line per workload."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK = 8.0e12


def summary(d, kernel=""):
    out = subprocess.run([sys.executable, os.path.join(HERE, "pmc_summary.py"), d, "--kernel",
                          kernel], capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def bench_line(log):
    with open(log) as f:
        for line in f:
            if line.startswith("{"):
                return json.loads(line)
    raise SystemExit(f"{log}: no bench line")


def one(o, kernel, field):
    res = {k: v for k, v in summary(o, kernel).items() if field in v}
    assert len(res) == 1, f"{o}: expected one kernel matching {kernel}, got {list(res)}"
    return next(iter(res.values()))[field]["mean"]


def main():
    o, wls = sys.argv[1], sys.argv[2:]
    known = 1283291200.0  # tools/pmc_calibrate.py: every B row gathered once (profiles/traffic.json)
    factor = known / (one(os.path.join(o, "cfetch"), "csr_mergepath_kernel", "FETCH_SIZE") * 1024)
    for wl in wls:
        b = bench_line(os.path.join(o, f"kt_{wl}.log"))
        rf = b["roofline"]
        key = rf.get("traffic_key") or {"workload": wl}
        kname = key.get("kernel", rf["kernel"]).split("<")[0].split(" ")[0]
        dur = one(os.path.join(o, f"kt_{wl}"), kname, "duration_ns") * 1e-9
        fetch = one(os.path.join(o, f"fetch_{wl}"), kname, "FETCH_SIZE") * 1024
        write = one(os.path.join(o, f"write_{wl}"), kname, "WRITE_SIZE") * 1024
        hbm = fetch * factor + write
        model = rf.get("bytes_per_launch") or rf.get("algorithmic_bytes_per_launch")
        # the bench line's lookup key (workload, kernel, K, dtype, nnzb, variant,
        # kernel source tag): bench.py uses these bytes only for that exact run shape
        print(json.dumps({
            **key, "kernel_trace_ms": round(dur * 1e3, 4),
            "bench_kernel_ms": rf.get("kernel_ms"),
            "fetch_size_bytes_raw": round(fetch), "fetch_correction": round(factor, 4),
            "write_size_bytes": round(write), "counter_bytes_per_launch": round(hbm),
            "counter_TBps": round(hbm / dur / 1e12, 3),
            "counter_frac_of_8TBps": round(hbm / dur / HBM_PEAK, 4),
            "model_bytes_per_launch": model,
            "model_frac": rf.get("frac"),
            "model_over_counter": round(model / hbm, 3) if model else None,
            "upper_model_bytes": rf.get("bytes_model_upper")}))


if __name__ == "__main__":
    main()
