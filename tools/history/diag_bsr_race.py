"""Diagnostic for an intermittent bs = 32 BSR mismatch at reddit scale
(tests/test_gpu_scale.py): repeats the CSR and BSR products on the same
inputs and prints where repeated runs disagree (which kernel, which rows /
columns / block rows). GPU box only; tuning/diagnostic, not a test.

usage: python tools/diag_bsr_race.py [reps]   (SPMM_BSR_VARIANT picks a kernel)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "spmm-denseblock_amd"))
from spmm_hip import ops, prep  # noqa: E402


def report(tag, got, ref, absd, tol=2e-5, explain=None):
    err = (got - ref).abs()
    bad = (err > tol * absd + 1e-30).nonzero()
    if bad.numel() == 0:
        return 0
    rows = bad[:, 0].cpu().numpy()
    cols = bad[:, 1].cpu().numpy()
    print(f"  {tag}: {len(rows)} bad, rows {np.unique(rows)[:8]} (block rows "
          f"{np.unique(rows // 32)[:8]}), cols {np.unique(cols)[:40]}, max err "
          f"{float(err.max()):.4g}", flush=True)
    if explain is not None:
        rp, ci, v, B = explain
        e = (got - ref).cpu().numpy()
        for r in np.unique(rows)[:4]:
            bc = np.sort(cols[rows == r])
            runs, st = [], bc[0]
            for a, b in zip(bc[:-1], bc[1:]):
                if b != a + 1:
                    runs.append((st, a)); st = b
            runs.append((st, bc[-1]))
            lo, hi = rp[r], rp[r + 1]
            Bn = B.cpu().numpy()
            best = None
            for q in range(lo, hi):
                c = ci[q]
                res = np.abs(e[r, bc] + v[q] * Bn[c, bc]).max()
                if best is None or res < best[0]:
                    best = (res, c, v[q])
            print(f"    row {r}: bad col runs {runs}; best missing-term fit: col {best[1]} "
                  f"(block col {best[1] // 32}, in-block col {best[1] % 32}), a={best[2]:.4f}, "
                  f"residual {best[0]:.3g} vs max err {np.abs(e[r, bc]).max():.3g}", flush=True)
    return len(rows)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    n, K, bs = 232965, 128, 32
    rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = [torch.from_numpy(a).to(dev) for a in (rp, ci, v)]
    mb = (n + bs - 1) // bs
    torch.manual_seed(0)
    B = torch.rand((mb * bs, K), device=dev) * 2 - 1
    Bn = B[:n].contiguous()
    Cc = ops.gespmm_csrmm(drp, dci, dv, Bn)
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), Bn.abs())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    Cb0 = torch.empty((mb * bs, K), device=dev)
    ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb0, ldc=K)
    torch.cuda.synchronize()
    print("variant", os.environ.get("SPMM_BSR_VARIANT", "default"), "nnzb", bci.numel(), flush=True)
    tot_b = tot_c = 0
    tot_b += report("bsr run 0 vs csr", Cb0[:n], Cc, absd)
    for i in range(reps):
        Cb = torch.empty((mb * bs, K), device=dev)
        ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb, ldc=K)
        C2 = ops.gespmm_csrmm(drp, dci, dv, Bn)
        torch.cuda.synchronize()
        nb = int((Cb != Cb0).sum())
        nc = int((C2 != Cc).sum())
        print(f"rep {i}: bsr differs from bsr run 0 in {nb}, csr from csr run 0 in {nc}", flush=True)
        tot_b += report("bsr vs csr", Cb[:n], Cc, absd, explain=(rp, ci, v, B))
        if nc:
            tot_c += report("csr vs csr run 0", C2, Cc, absd)
    print(f"total bad: bsr {tot_b}, csr {tot_c}", flush=True)


if __name__ == "__main__":
    main()
