"""Child process of tests/test_gpu_configs.py::test_config4_torch_distributed_world1.

torch.distributed with backend "nccl" (RCCL on ROCm) at world 1, initialised
before any GPU call of this process, then BASELINE config 4's exchange path of
bench.py on a power-law graph:

* chunks = 1: the rank's rows into its slot of the padded buffer, then the
  in-place all_gather_into_tensor (spmm_hip.dist.gather) — bit-identical to
  the whole-matrix call (one shard = the whole matrix, same kernel launch);
* chunks = 4: spmm_hip.dist.chunked_spmm, each chunk's all-gather issued
  async_op on RCCL's stream while the next chunk computes — within the fp32
  bar of the whole-matrix call (a chunk boundary splits merge-path rows
  differently);
* the exchange alone (4 async all-gathers) timed over 20 repetitions.

Prints one JSON line; the parent asserts on it.
"""
from __future__ import annotations

import json
import os
import sys
import time

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
    # chunks = 1: kernel into the slot, in-place all-gather
    out1 = torch.full((shard.max_rows, K), float("nan"), device=dev)
    ops.csrmm(drp, dci, dv, B, m=shard.rows, n=K, k=n, ldb=K, C=out1[:shard.rows], ldc=K,
              handle=h)
    C1 = sdist.gather(out1, shard, compact=True)
    torch.cuda.synchronize()
    res["chunks1_bit_identical"] = bool(torch.equal(C1, Cw))

    # chunks = 4: chunk c's async all-gather overlaps chunk c + 1's kernel
    nch = 4
    out = torch.full((nch, 1, sdist.chunk_rows(shard, nch), K), float("nan"), device=dev)

    def compute_chunk(r0, r1, dest):
        ops.csrmm(drp[r0:r1 + 1], dci, dv, B, m=r1 - r0, n=K, k=n, ldb=K, C=dest, ldc=K,
                  handle=h)

    C4 = sdist.chunked_spmm(shard, out, compute_chunk, nch, compact=True)
    torch.cuda.synchronize()
    err = (C4 - Cw).abs()
    res["chunks4_within_bar"] = bool((err <= 2e-5 * absd + 1e-30).all())
    res["chunks4_max_rel"] = float((err / (absd + 1e-30)).max())
    res["chunks4_no_nan"] = not bool(torch.isnan(C4).any())

    def exchange_only():
        works = [dist.all_gather_into_tensor(out[c].view(-1, K), out[c, 0], async_op=True)
                 for c in range(nch)]
        for w in works:
            w.wait()

    for _ in range(3):
        exchange_only()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        exchange_only()
    torch.cuda.synchronize()
    res["allgather_ms"] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
    res["allgather_bytes_per_call"] = int(out.numel() * 4)
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
