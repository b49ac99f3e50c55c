"""TUNING A/B helper (GPU box): the grouped bs 32 stream's k = 2 variant
(SPMM_GRP32_VARIANT=1033 in a TUNING build) against spmm_bsrmm_ex_f32 on a
column-sparse random matrix: max |diff| / (|A||B| row-column bound)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spmm-denseblock_amd"), os.path.join(ROOT, "tests")]
from spmm_hip import ops  # noqa: E402
from test_gpu_bsr import _column_sparse_bsr  # noqa: E402

rng = np.random.default_rng(7)
mb, kb, n = 301, 300, 128
rp, ci, v = _column_sparse_bsr(rng, mb, kb, 32, 0.3)
dev = torch.device("cuda:0")
drp, dci, dv = (torch.from_numpy(a).to(dev) for a in (rp, ci, v))
B = torch.rand((kb * 32, n), device=dev) * 2 - 1
C1 = torch.zeros((mb * 32, n), device=dev)
C2 = torch.zeros((mb * 32, n), device=dev)
ops.bsrmm(drp, dci, dv, B, mb=mb, kb=kb, n=n, bs=32, ldb=n, C=C1, ldc=n)
for W in (2, 4):
    g = ops.GroupedBsr32(drp, dci, dv, mb=mb, group_rows=W)
    g.mm(B, kb=kb, n=n, ldb=n, C=C2, ldc=n)
    torch.cuda.synchronize()
    Ab = ops.bsrmm(drp, dci, dv.abs(), B.abs(), mb=mb, kb=kb, n=n, bs=32, ldb=n,
                   C=torch.zeros_like(C1), ldc=n)
    err = float(((C2 - C1).abs() / Ab.clamp_min(1e-30)).max())
    print(f"W={W} max normwise error {err:.3e}  equal={bool(torch.equal(C1, C2))}", flush=True)
    assert err < 1e-5, err
    g.close()
