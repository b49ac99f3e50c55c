#!/usr/bin/env python3
"""Known-byte calibration run for the PMC traffic counters.

A permutation-matrix SpMM with the bench's shape (n = 2,449,029, K = 128)
reads every B row exactly once with the same 512-byte, dwordx2-per-lane
gathers as the real workload, so its HBM bytes are known:
  reads  = B (4*K*n) + colind + val (8*n) + rowptr (4*(n+1))
  writes = C (4*K*n) + carries (negligible)
FETCH_SIZE / WRITE_SIZE of this run against those bytes give the correction
factors applied to the bench's counters (tools/pmc_summary.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spmm_hip import ops  # noqa: E402

n, K = 2449029, 128
perm = np.random.default_rng(5).permutation(n).astype(np.int32)
rp = torch.arange(n + 1, dtype=torch.int32, device="cuda")
ci = torch.from_numpy(perm).cuda()
v = torch.ones(n, dtype=torch.float32, device="cuda")
B = torch.rand((n, K), device="cuda")
C = torch.empty((n, K), device="cuda")
# evict: stream a 1 GiB buffer between launches so B is not cache-resident
junk = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
h = ops.Handle()
for _ in range(4):
    junk.fill_(1.0)
    ops.csrmm(rp, ci, v, B, n=K, k=n, ldb=K, C=C, ldc=K, handle=h)
torch.cuda.synchronize()
assert torch.equal(C[0], B[perm[0]].float())
print({"calib_reads": 4 * K * n + 8 * n + 4 * (n + 1), "calib_writes": 4 * K * n})
