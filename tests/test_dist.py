"""Multi-rank plumbing of the row-partitioned path on CPU with
gloo, world_size 2 and 3: nnz-balanced sharding, the exact-shard exchange
into the contiguous [m, K] C (batched isend / irecv, chunked), and the
gathered C equal to the single-process result bit for bit. The per-shard
compute is injected (the oracle, test infrastructure) — on the GPU box the
same code runs the HIP kernel with RCCL."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "spmm-denseblock_amd"), os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    from helpers import load_oracle, oracle_csrmm_f32
    from spmm_hip import dist as sdist
    from spmm_hip import prep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = load_oracle()
        n, nnz, K = 5000, 60000, 24
        rp, ci = prep.powerlaw_csr(n, nnz, 900, 2.3, 11)
        val = np.random.default_rng(1).uniform(-1, 1, nnz).astype(np.float32)
        B = np.random.default_rng(2).uniform(-1, 1, (n, K)).astype(np.float32)
        sh = sdist.make_shard(rp, ci, val, rank, world)

        def compute(shard, Bt, rows):
            c = oracle_csrmm_f32(L, shard.rows, K, shard.rowptr, shard.colind, shard.val,
                                 Bt.numpy(), K, 0)
            rows.copy_(torch.from_numpy(c.reshape(shard.rows, K)))

        out = torch.full((n, K), float("nan"))
        C = sdist.partitioned_spmm(sh, torch.from_numpy(B), out, compute)
        full = oracle_csrmm_f32(L, n, K, rp, ci, val, B, K, 0).reshape(n, K)
        ok = bool(np.array_equal(C.numpy(), full)) and C.data_ptr() == out.data_ptr()
        try:  # a padded or short C is refused before anything moves
            sdist.gather(torch.zeros((n + 1, K)), sh)
            ok = False
        except ValueError:
            pass

        # chunked exchange: chunk c's all-gather in flight while c+1 computes
        def compute_chunk(r0, r1, dest):
            lrp = (sh.rowptr[r0:r1 + 1] - sh.rowptr[r0]).astype(np.int32)
            j0, j1 = int(sh.rowptr[r0]), int(sh.rowptr[r1])
            c = oracle_csrmm_f32(L, r1 - r0, K, lrp, sh.colind[j0:j1], sh.val[j0:j1],
                                 B, K, 0)
            dest.copy_(torch.from_numpy(c.reshape(r1 - r0, K)))

        # 64 chunks: the ranks' row counts differ (nnz-balanced bounds), so the
        # shorter ranks' trailing chunks are empty (skipped on both sides)
        assert any(sdist.chunk_range(sh, r, 63, 64)[0] == sdist.chunk_range(sh, r, 63, 64)[1]
                   for r in range(world))
        for nch in (1, 3, 7, 64):
            buf = torch.full((n, K), float("nan"))
            Cc = sdist.chunked_spmm(sh, buf, compute_chunk, nch)
            ok = ok and bool(np.array_equal(Cc.numpy(), full))
        q.put((rank, ok, sh.bounds.tolist(), sh.nnz))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_partitioned_allgather_matches_single(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    nnzs = [z for *_, z in res]
    assert sum(nnzs) == 60000
    assert max(nnzs) - min(nnzs) <= 900 + 5000 // world  # balanced within a row + rows share


def test_stacked_block_weak_scaling_graph():
    """bench.py's weak-scaling input (spmm_hip.dist.stacked_block): world = 1
    is the 1-GPU graph itself; at world > 1 block r keeps its generator's row
    structure, its columns map back to the 1-GPU columns by // world, rows stay
    sorted, ids span the world*n-row B, and blocks differ between ranks."""
    sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))
    from spmm_hip import dist as sdist
    from spmm_hip import prep
    n, nnz, md = 3000, 40000, 700
    rp1, ci1 = prep.powerlaw_csr(n, nnz, md, 2.3, 1234)
    rp, ci = sdist.stacked_block(n, nnz, md, 0, 1)
    assert np.array_equal(rp, rp1) and np.array_equal(ci, ci1)
    for world in (2, 8):
        blocks = []
        for r in range(world):
            base_rp, base_ci = prep.powerlaw_csr(n, nnz, md, 2.3, 1234 + r)
            rp, ci = sdist.stacked_block(n, nnz, md, r, world)
            assert ci.dtype == np.int32 and rp.dtype == np.int32
            assert np.array_equal(rp, base_rp) and ci.size == nnz
            assert np.array_equal(ci // world, base_ci)
            assert ci.min() >= 0 and ci.max() < world * n
            d = np.diff(ci.astype(np.int64))
            starts = np.zeros(nnz, bool)
            starts[rp[:-1][np.diff(rp) > 0]] = True
            assert np.all(d[~starts[1:]] >= 0), "rows must stay sorted"
            blocks.append(ci)
        # a column shared by two blocks lands on different B rows in each
        for r in range(1, world):
            m0 = dict(zip((blocks[0] // world).tolist(), blocks[0].tolist()))
            shared = [(c, x) for c, x in zip((blocks[r] // world).tolist(), blocks[r].tolist())
                      if c in m0]
            assert shared and all(m0[c] != x for c, x in shared)
