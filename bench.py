#!/usr/bin/env python3
"""bench.py — BASELINE.json headline: SpMM GFLOP/s (2*nnz*K/t) + achieved HBM
GB/s on ogbn-products at K = 128 (synthetic stand-in of the same n / nnz /
max degree: the dataset is not reachable offline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--K 128]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one pass of the hot path over the resident inputs: the CSR x dense
SpMM (merge-path kernel + carry fix-up) on this rank's rows, and for N > 1
the RCCL all-gather of C (BASELINE config 4, strong scaling: the total graph
is fixed, rows are split nnz-balanced). Inputs are in HBM before timing
starts. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
PRODUCTS = dict(n=2449029, nnz=61859140, max_deg=17481, gamma=2.3)


def algorithmic_bytes(n_rows: int, nnz: int, K: int) -> int:
    """SURVEY.md §8(d) CSR gather model: rowptr + (colind, val) + one B row
    per nnz + the C write."""
    return 4 * (n_rows + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n_rows


def cpu_baseline(rp: np.ndarray, ci: np.ndarray, K: int, budget_s: float = 12.0) -> dict:
    """spmm.cc csr_spmm restated (oracle_spmm_cc_csr: OpenMP rows, k-outer,
    double, unit values) timed on a growing row prefix of the SAME graph
    until ~budget_s of CPU work; reports GFLOP/s = 2*nnz_sample*K/t."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import load_oracle, ptr
    L = load_oracle()
    n = rp.size - 1
    Bd = np.random.default_rng(1).uniform(-1, 1, (n, K))  # double, as spmm.cc
    ip64 = rp.astype(np.int64)
    ix64 = ci.astype(np.int64)
    rows = 1024
    best = None
    while True:
        rows = min(rows, n)
        out = np.empty((rows, K))
        t0 = time.perf_counter()
        L.oracle_spmm_cc_csr(rows, K, ptr(ip64), ptr(ix64), ptr(Bd), K, ptr(out))
        dt = time.perf_counter() - t0
        nnz_s = int(rp[rows])
        best = dict(rows=rows, nnz=nnz_s, seconds=dt)
        if dt >= budget_s / 4 or rows == n:
            break
        rows = int(rows * min(8.0, max(2.0, (budget_s / 4) / max(dt, 1e-4))))
    g = 2.0 * best["nnz"] * K / best["seconds"] / 1e9
    return {"value": round(g, 3), "unit": "GFLOP/s", "cores": int(L.oracle_num_threads()),
            "kind": "port",
            "sample": (f"spmm.cc csr_spmm restated (double, unit values, k-outer) on the first "
                       f"{best['rows']} rows ({best['nnz']} nnz) of the same synthetic "
                       f"ogbn-products graph, K={K}, {best['seconds']:.2f} s")}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (profiles/, see DESIGN.md §7)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from spmm_hip import dist as sdist
    from spmm_hip import ops, prep

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    K = args.K
    P = PRODUCTS
    t_gen = time.perf_counter()
    rp, ci = prep.powerlaw_csr(P["n"], P["nnz"], P["max_deg"], P["gamma"], 1234)
    val = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    t_gen = time.perf_counter() - t_gen
    n, nnz = rp.size - 1, ci.size

    shard = sdist.make_shard(rp, ci, val, rank, world)
    d_rp = torch.from_numpy(shard.rowptr).to(dev)
    d_ci = torch.from_numpy(np.ascontiguousarray(shard.colind)).to(dev)
    d_v = torch.from_numpy(np.ascontiguousarray(shard.val)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    B = torch.rand((n, K), device=dev, generator=g) * 2 - 1
    out = torch.empty((world * shard.max_rows, K), device=dev)
    mr = shard.max_rows
    C_slot = out[rank * mr: rank * mr + shard.rows]

    h = ops.Handle()
    if args.waves_per_cu:
        h.set_csr_waves_per_cu(args.waves_per_cu)
    local_nnz = int(shard.colind.size)

    def step():
        ops.csrmm(d_rp, d_ci, d_v, B, m=shard.rows, n=K, k=n, ldb=K, C=C_slot, ldc=K, handle=h)
        if world > 1:
            sdist.gather(out, shard, compact=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    h.kernel_times()  # drop warm-up records
    h.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    h.set_timing(False)
    ktimes = h.kernel_times()
    kms = float(np.mean(ktimes)) if ktimes else float("nan")

    # max over ranks
    t = torch.tensor([elapsed, kms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kms_max = float(t[0]), float(t[1])

    ms_step = elapsed / args.steps * 1e3
    flops = 2.0 * nnz * K
    value = flops * args.steps / elapsed / 1e9
    # dominant kernel = rank-local merge-path SpMM launch
    kbytes = algorithmic_bytes(shard.rows, local_nnz, K)
    achieved = kbytes / (kms / 1e3) / 1e9 if ktimes else None
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("K") == K and tj.get("nnz") == local_nnz:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(rp, ci, K)
        rec = {
            "metric": "SpMM GFLOP/s (2*nnz*K/t) + achieved HBM GB/s, ogbn-products K=128",
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (Chung-Lu power-law graph with ogbn-products n/nnz/max-degree, "
                    "U(-1,1) values and B; OGB data not reachable offline)",
            "config": {"workload": "csr_spmm ogbn-products-synthetic K=%d%s" %
                                   (K, " row-partitioned + RCCL all-gather" if world > 1 else ""),
                       "n": n, "nnz": nnz, "K": K, "max_deg": int(np.diff(rp).max()),
                       "parallelism": f"rows{world}" if world > 1 else "single",
                       "waves_per_cu": args.waves_per_cu or 16},
            "roofline": {"bound": "hbm",
                         "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                         "traffic": traffic,
                         "kernel": "csr_mergepath_kernel<2>",
                         "kernel_ms": round(kms, 4), "kernel_ms_max_rank": round(kms_max, 4),
                         "algorithmic_bytes_per_launch": kbytes},
            "cpu_baseline": cpu,
            "gen_seconds": round(t_gen, 2),
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
