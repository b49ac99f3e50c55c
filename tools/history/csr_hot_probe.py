"""Probe: the CSR merge-path kernel with hot-column cache hints (spmm_csrmm_hot_f32).

Products stand-in (bench.py's products_csr, K = 128). The H columns with the
most nonzeros keep the default cache policy for their B-row gathers; every
other B row is gathered non-temporal (nt). H = 0 streams every row; "plain" is
the shipped kernel (no tags). The tags come from the device analysis
(spmm_csr_hot_analysis), checked against the host's column counts. Prints per-H kernel ms (HIP events, median of
launches) and checks C bit-identical to the plain kernel (same FMA order).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))


def main():
    import torch
    from spmm_hip import ops, prep
    K = int(os.environ.get("K", "128"))
    Hs = [int(x) for x in os.environ.get("HS", "0 4096 8192 16384 65536 262144 1048576").split()]
    reps = int(os.environ.get("REPS", "20"))
    dev = torch.device("cuda", 0)
    rp, ci = prep.powerlaw_csr(2449029, 61859140, 17481, 2.3, 1234)
    val = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    n = rp.size - 1
    cnt = np.bincount(ci, minlength=n)
    order = np.argsort(-cnt, kind="stable")
    d_rp = torch.from_numpy(rp).to(dev)
    d_v = torch.from_numpy(val).to(dev)
    d_ci = torch.from_numpy(ci).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    B = torch.rand((n, K), device=dev, generator=g) * 2 - 1
    C = torch.empty((n, K), device=dev)
    h = ops.Handle()

    def run(colind, flags, hot):
        h.set_csr_options(flags)
        f = ops.csrmm_hot if hot else ops.csrmm
        for _ in range(3):
            f(d_rp, colind, d_v, B, m=n, n=K, k=n, ldb=K, C=C, ldc=K, handle=h)
        torch.cuda.synchronize()
        h.kernel_times()
        h.set_timing(True)
        for _ in range(reps):
            f(d_rp, colind, d_v, B, m=n, n=K, k=n, ldb=K, C=C, ldc=K, handle=h)
        torch.cuda.synchronize()
        h.set_timing(False)
        return float(np.median(h.kernel_times()))

    ref_ms = run(d_ci, 1, False)
    Cref = C.clone()
    tagged = {}
    for H in Hs:
        # device analysis (spmm_csr_hot_analysis), hot_bytes = H rows of K floats
        t = ops.csr_hot_analysis(d_ci, n=K, k=n, hot_bytes=H * 4 * min(K, 256) if H else 4,
                                 handle=h)
        torch.cuda.synchronize()
        # the host reference of the same selection: the columns with the most
        # nonzeros, ties at the threshold count left out
        tags = (t < 0).cpu().numpy()
        if not np.array_equal(t.cpu().numpy() & 0x7fffffff, ci):
            raise SystemExit("analysis changed an index")
        hot_cols = np.unique(ci[tags])
        if hot_cols.size > max(H, 1) or (hot_cols.size and cnt[hot_cols].min() <
                                         cnt[np.setdiff1d(np.arange(n), hot_cols)].max(initial=0)):
            raise SystemExit(f"analysis hot set wrong: {hot_cols.size} columns for H={H}")
        tagged[H] = (t, float(tags.mean()), int(hot_cols.size))
    res = []
    for rnd in range(2):
        res.append({"H": "plain", "ms": run(d_ci, 1, False)})
        for H in Hs:
            ms = run(tagged[H][0], 1, True)
            same = bool(torch.equal(C, Cref))
            res.append({"H": H, "hot_cols": tagged[H][2], "hot_nnz_frac": round(tagged[H][1], 4),
                        "ms": round(ms, 4), "bit_identical": same})
            print(json.dumps(res[-1]), flush=True)
            if not same:
                raise SystemExit("HOT kernel differs from the plain kernel")
        print(json.dumps(res[-len(Hs) - 1]), flush=True)
    print(json.dumps({"plain_first_ms": round(ref_ms, 4), "K": K}))


if __name__ == "__main__":
    main()
