"""Bit-for-bit comparison of bs 16 fp16 kernels on the products stand-in
(community order, K = 512): run once per SPMM_BSR_VARIANT (the variant is read
once per process) and print a digest of C. The item stream (55PR / 56PR) sums
the same items in the same order as the column stream (5021), so the digests
must agree. GPU box only; diagnostic, not a test.

usage: SPMM_BSR_VARIANT=<v> python tools/is16_check.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "spmm-denseblock_amd"))
from spmm_hip import ops, prep  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, bs, K = 2449029, 16, 512
    rp, ci = prep.community_csr(n, 27.0, 32, 512, 0.97, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = [torch.from_numpy(a).to(dev) for a in (rp, ci, v)]
    mb = (n + bs - 1) // bs
    torch.manual_seed(0)
    B16 = (torch.rand((mb * bs, K), device=dev) * 2 - 1).half()
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    bv16 = bval.half()
    del bval
    C = torch.empty((mb * bs, K), device=dev)
    digests = []
    for _ in range(3):
        C.fill_(float("nan"))
        ops.bsrmm_f16(brp, bci, bv16, B16, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K)
        torch.cuda.synchronize()
        digests.append(hashlib.sha1(C[:n].cpu().numpy().tobytes()).hexdigest()[:16])
    finite = bool(torch.isfinite(C[:n]).all())
    print(f"variant {os.environ.get('SPMM_BSR_VARIANT', 'default')} digests {digests} "
          f"finite {finite} sum {float(C[:n].double().sum()):.6f}", flush=True)


if __name__ == "__main__":
    main()
