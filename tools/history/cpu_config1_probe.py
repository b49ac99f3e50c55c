"""Probe: BASELINE config 1 (spmm.cc csr_spmm on randomCSRMatrix(16384, 16384,
2^-10), K = 32) under several OpenMP environments, each in a fresh process,
to see which gives per-sample spreads under 10 % on a CPU-quota'd host.

usage: python tools/cpu_config1_probe.py            (parent: runs the variants)
       python tools/cpu_config1_probe.py --child    (one variant, env from the parent)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))
    import bench
    from helpers import load_oracle
    res = bench.cpu_baseline_config1(load_oracle())
    c = res["csr_spmm"]
    print(json.dumps({"threads": res["cores"], "GFLOPs": c["GFLOPs"], "spread": c["spread"],
                      "min_s": c["min_s"], "median_s": c["median_s"], "max_s": c["max_s"],
                      "calls_per_sample": c["calls_per_sample"]}), flush=True)


def main():
    import bench
    hc = bench._host_cpus()
    P = hc["physical_cores_in_affinity"]
    print(json.dumps(hc), flush=True)
    variants = [
        ("protocol", {"OMP_NUM_THREADS": str(P), "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}),
        ("protocol+passive", {"OMP_NUM_THREADS": str(P), "OMP_PROC_BIND": "close",
                              "OMP_PLACES": "cores", "OMP_WAIT_POLICY": "passive"}),
        ("16+close", {"OMP_NUM_THREADS": "16", "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}),
        ("16+passive", {"OMP_NUM_THREADS": "16", "OMP_PROC_BIND": "close", "OMP_PLACES": "cores",
                        "OMP_WAIT_POLICY": "passive"}),
    ]
    for rep in range(2):
        for name, env in variants:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"],
                               env=dict(os.environ, **env), stdout=subprocess.PIPE, text=True,
                               timeout=300)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(json.dumps({"variant": name, "rep": rep, **(json.loads(lines[-1]) if lines else
                                                               {"error": r.returncode})}),
                  flush=True)


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    child() if "--child" in sys.argv else main()
