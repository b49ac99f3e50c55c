"""Child process of tests/test_gpu_configs.py::test_config4_torch_distributed_world1.

torch.distributed with backend "nccl" (RCCL on ROCm) at world 1, initialised
before any GPU call of this process, then BASELINE config 4's exchange path of
bench.py on a power-law graph:

* chunks = 1: spmm_hip.dist.partitioned_spmm, the rank's rows written in
  place into the contiguous n x K C — bit-identical to the whole-matrix call
  (one shard = the whole matrix, same kernel launch);
* chunks = 4: spmm_hip.dist.chunked_spmm — within the fp32 bar of the
  whole-matrix call (a chunk boundary splits merge-path rows differently);
* a world-1 rank has no peer: the exchange issues no request;
* bench.py's max-over-ranks timing all_reduce through RCCL.

Prints one JSON line; the parent asserts on it.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)  # before any other GPU call
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    torch.cuda.set_device(dev)
    from spmm_hip import dist as sdist
    from spmm_hip import ops, prep

    n, nnz, K = 400000, 8000000, 256
    rp, ci = prep.powerlaw_csr(n, nnz, 6000, 2.3, 99)
    v = np.random.default_rng(3).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = (torch.from_numpy(a).to(dev) for a in (rp, ci, v))
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    B = torch.rand((n, K), device=dev, generator=g) * 2 - 1
    h = ops.Handle()
    Cw = torch.empty((n, K), device=dev)
    ops.csrmm(drp, dci, dv, B, n=K, k=n, ldb=K, C=Cw, ldc=K, handle=h)
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B.abs())

    shard = sdist.make_shard(rp, ci, v, 0, 1)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    # chunks = 1: the kernel into the rank's rows of C, then the exchange
    C1 = torch.full((n, K), float("nan"), device=dev)

    def compute(sh, B_, rows):
        ops.csrmm(drp, dci, dv, B_, m=sh.rows, n=K, k=n, ldb=K, C=rows, ldc=K, handle=h)

    sdist.partitioned_spmm(shard, B, C1, compute)
    torch.cuda.synchronize()
    res["chunks1_bit_identical"] = bool(torch.equal(C1, Cw))

    # chunks = 4: chunk c's exchange would overlap chunk c + 1's kernel
    nch = 4
    C4 = torch.full((n, K), float("nan"), device=dev)

    def compute_chunk(r0, r1, dest):
        ops.csrmm(drp[r0:r1 + 1], dci, dv, B, m=r1 - r0, n=K, k=n, ldb=K, C=dest, ldc=K,
                  handle=h)

    sdist.chunked_spmm(shard, C4, compute_chunk, nch)
    torch.cuda.synchronize()
    err = (C4 - Cw).abs()
    res["chunks4_within_bar"] = bool((err <= 2e-5 * absd + 1e-30).all())
    res["chunks4_max_rel"] = float((err / (absd + 1e-30)).max())
    res["chunks4_no_nan"] = not bool(torch.isnan(C4).any())
    res["chunks4_bit_identical"] = bool(torch.equal(C4, Cw))
    res["exchange_requests_world1"] = len(sdist.exchange_chunk(C4, shard, 0, nch))
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res["allreduce_max_ok"] = t.tolist() == [1.5, 2.5]
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
