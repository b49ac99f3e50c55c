#!/usr/bin/env python3
"""The reference's own benchmark sweep (benchmark.py:3-31) on this build.

test_bsrmm (benchmark.py:3-19, test_bsrmm.cu:46-181): m = n = 2 << 16, a
uniform-random block pattern of block density p (Bernoulli(p) per block, as
randomBSRMatrix, load_data.cc:81-113), dense U(-1, 1) blocks, B dense; one
cusparseSbsrmm / rocsparse_bsrmm_template call with C column-major (ldc = m)
and transB = 0 (B column-major, ldb = n) or 1 (B row-major, ldb = dim).
Both of the reference's impls bind spmm_sbsrmm here (include/spmm_compat.hpp),
so one column serves both.

test_csrmm (benchmark.py:21-31, test_csrmm.cu:46-153): the same m = n, a
random CSR of density p (Bernoulli(p) per entry, as randomCSRMatrix,
load_data.cc:42-69), U(-1, 1) values; gespmm (gespmm_csrmm<float>: B and C
row-major) and cusparse (cusparseScsrmm: B and C column-major).

The patterns are drawn on the device with the same distribution (Binomial
row counts, uniform columns, duplicates dropped: 0.5 % fewer entries than
p at p = 2e-2), not from the reference's mt19937_64 stream: drawing 2^34
Bernoulli variables per CSR matrix on the host would take minutes per cell.
Each cell: 2 warm-up calls, then `--reps` calls each timed with hipEvents
(staging transposes included, as the reference times the call); the median
is reported with the reference's printed GFLOPs (nnzb * bs^2 * dim / t, no
factor 2; csr: 2 nnz dim / t as run_csrmm prints), the useful rate
2 nnz dim / t, the compulsory-byte fraction of 8 TB/s (A + indices once,
each distinct B row once, the C write) and the fp32 fraction of 157.3 TFLOP/s
(MFMA at bs >= 16; the VALU kernel at bs <= 8, whose own peak is the same
with packed FMAs).

    python tools/ref_sweep.py > sweep.jsonl 2> progress.log
    python tools/ref_sweep.py --table sweep.jsonl > table.md
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from ctypes import byref, c_float, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))

HBM = 8000.0
FP32_PEAK = 157.3
M = 2 << 16


def log(msg: str) -> None:
    print(f"[sweep {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def random_pattern(torch, rows: int, cols: int, p: float, gen):
    """(rowptr, colind) int32 on the device: Binomial(cols, p) entries per row at
    uniform distinct columns, sorted."""
    dev = gen.device
    cnt = torch.binomial(torch.full((rows,), float(cols), device=dev),
                         torch.full((rows,), float(p), device=dev), generator=gen).long()
    row = torch.repeat_interleave(torch.arange(rows, device=dev), cnt)
    col = torch.randint(cols, (row.numel(),), device=dev, generator=gen)
    key = torch.unique(row * cols + col)
    del row, col
    row, col = key // cols, key % cols
    rp = torch.zeros(rows + 1, dtype=torch.int32, device=dev)
    rp[1:] = torch.cumsum(torch.bincount(row, minlength=rows), 0).to(torch.int32)
    return rp, col.to(torch.int32)


def timed(torch, call, reps: int) -> list[float]:
    for _ in range(2):
        call()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        call()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b))
    return out


def bsr_cells(torch, lib, h, descr, p, bs, Ks, tbs, reps, gen):
    mb = nb = M // bs
    brp, bci = random_pattern(torch, mb, nb, p, gen)
    nnzb = int(bci.numel())
    val = torch.rand(nnzb * bs * bs, device=gen.device, generator=gen) * 2 - 1
    distinct_b_rows = int(torch.unique(bci).numel()) * bs
    one, zero = c_float(1.0), c_float(0.0)
    for K in Ks:
        Bt = torch.rand((M, K), device=gen.device, generator=gen) * 2 - 1  # row-major
        Bc = Bt.t().contiguous()                                            # column-major
        C = torch.empty((K, M), device=gen.device)                          # column-major
        for tb in tbs:
            Bx, ldb = (Bt, K) if tb else (Bc, M)

            def call():
                st = lib.spmm_sbsrmm(h.raw, 0, 0, tb, mb, K, nb, nnzb, byref(one), descr,
                                     c_void_p(val.data_ptr()), c_void_p(brp.data_ptr()),
                                     c_void_p(bci.data_ptr()), bs, c_void_p(Bx.data_ptr()), ldb,
                                     byref(zero), c_void_p(C.data_ptr()), M)
                if st != 0:
                    raise RuntimeError(f"spmm_sbsrmm status {st}")
            ts = sorted(timed(torch, call, reps))
            t = ts[len(ts) // 2]
            nnz = nnzb * bs * bs
            comp = 4 * (mb + 1) + 4 * nnzb + 4 * nnz + 4 * distinct_b_rows * K + 4 * M * K
            rec = {"kind": "bsrmm", "p": p, "bs": bs, "dim": K, "transB": tb, "nnzb": nnzb,
                   "block_density": round(nnzb / (mb * nb), 6), "ms": round(t, 4),
                   "ms_min": round(ts[0], 4), "ms_max": round(ts[-1], 4),
                   "ref_GFLOPs": round(nnzb / 1e6 * bs * bs * K / t, 1),
                   "useful_GFLOPs": round(2.0 * nnz * K / t / 1e6, 1),
                   "compulsory_bytes": comp,
                   "compulsory_frac": round(comp / (t / 1e3) / 1e9 / HBM, 4),
                   "fp32_frac": round(2.0 * nnz * K / (t / 1e3) / 1e12 / FP32_PEAK, 4),
                   "unit": "MFMA" if bs >= 16 else "VALU"}
            print(json.dumps(rec), flush=True)
            log(f"bsr p={p} bs={bs} K={K} tB={tb}: {t:.3f} ms, {rec['useful_GFLOPs']} GFLOP/s, "
                f"comp {rec['compulsory_frac']}, fp32 {rec['fp32_frac']}")
        del Bt, Bc, C
    del brp, bci, val


def csr_cells(torch, lib, h, descr, p, Ks, reps, gen):
    rp, ci = random_pattern(torch, M, M, p, gen)
    nnz = int(ci.numel())
    val = torch.rand(nnz, device=gen.device, generator=gen) * 2 - 1
    distinct = int(torch.unique(ci).numel())
    one, zero = c_float(1.0), c_float(0.0)
    for K in Ks:
        Bt = torch.rand((M, K), device=gen.device, generator=gen) * 2 - 1
        Bc = Bt.t().contiguous()
        C = torch.empty((M, K), device=gen.device)
        for impl in ("gespmm", "cusparse"):
            if impl == "gespmm":
                def call():
                    st = lib.spmm_gespmm_csrmm_f32(M, K, c_void_p(rp.data_ptr()),
                                                   c_void_p(ci.data_ptr()), c_void_p(val.data_ptr()),
                                                   c_void_p(Bt.data_ptr()), c_void_p(C.data_ptr()),
                                                   c_void_p(torch.cuda.current_stream().cuda_stream))
                    if st != 0:
                        raise RuntimeError(f"spmm_gespmm_csrmm_f32 status {st}")
            else:
                def call():
                    st = lib.spmm_scsrmm(h.raw, 0, M, K, M, nnz, byref(one), descr,
                                         c_void_p(val.data_ptr()), c_void_p(rp.data_ptr()),
                                         c_void_p(ci.data_ptr()), c_void_p(Bc.data_ptr()), M,
                                         byref(zero), c_void_p(C.data_ptr()), M)
                    if st != 0:
                        raise RuntimeError(f"spmm_scsrmm status {st}")
            ts = sorted(timed(torch, call, reps))
            t = ts[len(ts) // 2]
            gather = 4 * (M + 1) + 8 * nnz + 4 * K * nnz + 4 * K * M
            comp = 4 * (M + 1) + 8 * nnz + 4 * K * distinct + 4 * K * M
            rec = {"kind": "csrmm", "p": p, "dim": K, "impl": impl, "nnz": nnz, "ms": round(t, 4),
                   "ms_min": round(ts[0], 4), "ms_max": round(ts[-1], 4),
                   "GFLOPs": round(2.0 * nnz * K / t / 1e6, 1),
                   "gather_model_GBps": round(gather / (t / 1e3) / 1e9, 1),
                   "compulsory_frac": round(comp / (t / 1e3) / 1e9 / HBM, 4)}
            print(json.dumps(rec), flush=True)
            log(f"csr p={p} K={K} {impl}: {t:.3f} ms, {rec['GFLOPs']} GFLOP/s")
        del Bt, Bc, C
    del rp, ci, val


def table(path: str) -> None:
    """Markdown tables of a sweep's JSON lines: per (p, bs) the ms and useful GFLOP/s
    per dim (transB = 1 / 0), the compulsory-byte and fp32 fractions at dim 512; the
    CSR cells per (p, impl)."""
    rows = [json.loads(ln) for ln in open(path) if ln.startswith("{")]
    bsr = {(r["p"], r["bs"], r["dim"], r["transB"]): r for r in rows if r["kind"] == "bsrmm"}
    dims = sorted({k[2] for k in bsr})
    print("test_bsrmm (benchmark.py:3-19): ms, transB = 1 / 0; useful GFLOP/s (transB = 1); "
          "at dim 512: compulsory-byte fraction of 8 TB/s and fp32 fraction of 157.3 TFLOP/s\n")
    print("| p | bs | nnzb | " + " | ".join(f"dim {d}" for d in dims) +
          " | comp 512 | fp32 512 |")
    print("|" + "---|" * (len(dims) + 5))
    for p, bs in sorted({(k[0], k[1]) for k in bsr}):
        cells = []
        for d in dims:
            a, b = bsr.get((p, bs, d, 1)), bsr.get((p, bs, d, 0))
            cells.append(f"{a['ms']:.3f} / {b['ms']:.3f} ({a['useful_GFLOPs'] / 1e3:.1f} T)"
                         if a and b else "-")
        z = bsr.get((p, bs, dims[-1], 1), {})
        nz = next(r["nnzb"] for k, r in bsr.items() if k[:2] == (p, bs))
        print(f"| {p:g} | {bs} | {nz} | " + " | ".join(cells) +
              f" | {z.get('compulsory_frac', '-')} | {z.get('fp32_frac', '-')} |")
    csr = [r for r in rows if r["kind"] == "csrmm"]
    if csr:
        print("\ntest_csrmm (benchmark.py:21-31): ms (GFLOP/s), gespmm = row-major B and C, "
              "cusparse = column-major B and C\n")
        print("| p | impl | nnz | " + " | ".join(f"dim {d}" for d in dims) + " |")
        print("|" + "---|" * (len(dims) + 3))
        for p, impl in sorted({(r["p"], r["impl"]) for r in csr}):
            rr = {r["dim"]: r for r in csr if r["p"] == p and r["impl"] == impl}
            nz = next(iter(rr.values()))["nnz"]
            print(f"| {p:g} | {impl} | {nz} | " + " | ".join(
                f"{rr[d]['ms']:.3f} ({rr[d]['GFLOPs'] / 1e3:.2f} T)" if d in rr else "-"
                for d in dims) + " |")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--densities", default="0.0002,0.002,0.02")
    ap.add_argument("--bs", default="2,4,8,16,32,64")
    ap.add_argument("--dims", default="64,128,256,512")
    ap.add_argument("--transB", default="0,1")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--skip-csr", action="store_true")
    ap.add_argument("--skip-bsr", action="store_true")
    ap.add_argument("--table", default=None, help="print the markdown tables of a sweep JSONL")
    ap.add_argument("--bsr-options", type=int, default=0,
                    help="spmm_set_bsr_options flags of the handle (1: dense-block product)")
    args = ap.parse_args()
    if args.table:
        table(args.table)
        return
    import torch
    from spmm_hip import ops
    from spmm_hip._lib import lib
    L = lib()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    h = ops.Handle()
    if args.bsr_options:
        h.set_bsr_options(args.bsr_options)
    d = c_void_p()
    assert L.spmm_create_mat_descr(byref(d)) == 0
    Ks = [int(x) for x in args.dims.split(",")]
    dens = [float(x) for x in args.densities.split(",")]
    if not args.skip_bsr:
        for p in dens:
            for bs in (int(x) for x in args.bs.split(",")):
                bsr_cells(torch, L, h, d, p, bs, Ks, [int(x) for x in args.transB.split(",")],
                          args.reps, gen)
    if not args.skip_csr:
        for p in dens:
            csr_cells(torch, L, h, d, p, Ks, args.reps, gen)
    L.spmm_destroy_mat_descr(d)
    h.close()


if __name__ == "__main__":
    main()
