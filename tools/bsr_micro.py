#!/usr/bin/env python3
"""BSR bs=32 fp32 kernel micro-benchmark: the same block count with B panels
that stay in L2 ("hot": every block row uses the same few column blocks)
versus panels spread over the whole matrix ("cold"), to separate the
kernel's own ceiling from the memory system's. Prints MFMA TFLOP/s."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "spmm-denseblock_amd"))
from spmm_hip import ops  # noqa: E402

dev = torch.device("cuda", 0)
mb, per, bs, K = 8192, 64, 32, int(os.environ.get("K", "128"))
direction = int(os.environ.get("DIR", "0"))  # 0 = ROW blocks, 1 = COLUMN blocks
modes = (("hot", 8), ("warm", 256), ("cold", mb))
only = os.environ.get("MODE")
for mode, ncols in modes:
    if only and mode != only:
        continue
    rng = np.random.default_rng(0)
    cols = np.stack([np.sort(rng.choice(ncols, min(per, ncols), replace=False)) if ncols >= per
                     else np.sort(rng.choice(ncols, per, replace=True)) for _ in range(mb)])
    if ncols < per:  # duplicates allowed as separate blocks
        pass
    rp = torch.arange(0, mb * per + 1, per, dtype=torch.int32, device=dev)
    ci = torch.from_numpy(cols.reshape(-1).astype(np.int32)).to(dev)
    val = torch.rand(mb * per * bs * bs, device=dev)
    B = torch.rand(mb * bs, K, device=dev)
    C = torch.empty(mb * bs, K, device=dev)
    h = ops.Handle()
    for _ in range(3):
        ops.bsrmm(rp, ci, val, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K, handle=h,
                  direction=direction)
    torch.cuda.synchronize()
    h.kernel_times()
    h.set_timing(True)
    for _ in range(10):
        ops.bsrmm(rp, ci, val, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K, handle=h,
                  direction=direction)
    torch.cuda.synchronize()
    kt = float(np.mean(h.kernel_times()))
    fl = 2.0 * mb * per * bs * bs * K
    print(f"{mode:5s} dir={direction} var={os.environ.get('SPMM_BSR_VARIANT', 'default')} K={K} "
          f"{kt:.4f} ms {fl / kt / 1e9:.1f} TFLOP/s ({fl / kt / 1e9 / 157.3:.3f} of peak)", flush=True)
