#!/usr/bin/env python3
"""Column fill vs kernel (the panel probe's threshold): uniform-random bs 32 BSR
(4,096 block rows, 60 blocks each) whose blocks hold F of 32 nonzero columns, dim 64 / 128,
column-major C (the sweep's call); run once per library (LIBS: paths of builds that force the
column stream or the panel stream). One JSON line per (library, F, dim)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))


def main():
    import torch
    from spmm_hip import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    mb, per_row = 4096, 60
    ci = torch.sort(torch.rand((mb, mb), device=dev, generator=g).argsort(dim=1)[:, :per_row],
                    dim=1)[0].to(torch.int32).reshape(-1).contiguous()
    rp = torch.arange(0, mb * per_row + 1, per_row, dtype=torch.int32, device=dev)
    nnzb = ci.numel()
    for F in (4, 8, 12, 16, 20, 24, 28, 32):
        v = (torch.rand((nnzb, 32, 32), device=dev, generator=g) * 2 - 1)
        keep = torch.rand((nnzb, 32), device=dev, generator=g).argsort(dim=1) < F  # F columns
        v = (v * keep[:, None, :]).reshape(-1).contiguous()
        for K in (64, 128):
            B = torch.rand((mb * 32, K), device=dev, generator=g) * 2 - 1
            C = torch.empty(K * mb * 32, device=dev)
            call = lambda: ops.bsrmm(rp, ci, v, B, mb=mb, kb=mb, n=K, bs=32, ldb=K, C=C,
                                     ldc=mb * 32, order_c=ops.ORDER_COL)
            for _ in range(2):
                call()
            ts = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); call(); e1.record(); torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            print(json.dumps({"lib": os.environ.get("TAG", ""), "F": F, "dim": K,
                              "ms": round(ts[3], 4)}), flush=True)
        del v


if __name__ == "__main__":
    main()
