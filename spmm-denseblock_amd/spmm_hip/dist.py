"""Row-partitioned multi-GPU SpMM (BASELINE config 4).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).
Every rank holds the full dense B (replicated: 2.5 GB for products at K=256,
far under 288 GB), owns a contiguous nnz-balanced row range of A, computes
its rows of C with the HIP kernel, and the ranks exchange C with ONE
all-gather over xGMI. Output rows are independent: a row that no merge-path
wave splits is bit-identical to the 1-GPU result; a split row's carries are
associated by where the wave boundaries fall (within the fp32 bar).

Shards have unequal row counts; the all-gather runs on a padded
[world, max_rows, K] buffer whose rank-r slot is written in place by the
kernel (no staging copy). ``gather(..., compact=True)`` returns the dense
[m, K] matrix (one extra device copy); the padded buffer plus ``bounds`` is
the zero-copy form.

``chunked_spmm`` overlaps the exchange with the compute: each rank's rows are
cut into ``nchunks`` pieces, and piece c's all-gather (RCCL on its own
stream, ``async_op``) runs while piece c+1 is computed. The buffer is
chunk-major, [nchunks, world, rows_per_chunk, K], so every piece's gather is
one contiguous in-place all-gather.

``stacked_block`` is the weak-scaling form (bench.py's default at N > 1):
every rank owns a products-size row block of a world-times larger graph, B
replicated, and C stays row-sharded where the kernel wrote it — no
collective on the data path, per-GPU work fixed as N grows.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np

from . import prep


@dataclass
class Shard:
    rank: int
    world: int
    bounds: np.ndarray      # [world+1] row bounds (nnz-balanced)
    row0: int
    row1: int
    rowptr: np.ndarray      # local CSR, rebased to 0
    colind: np.ndarray
    val: np.ndarray

    @property
    def rows(self) -> int:
        return self.row1 - self.row0

    @property
    def max_rows(self) -> int:
        return int(np.max(np.diff(self.bounds)))


def make_shard(rowptr: np.ndarray, colind: np.ndarray, val: np.ndarray, rank: int,
               world: int) -> Shard:
    """Cut rank's row range out of a global CSR (host side)."""
    bounds = prep.partition_rows(rowptr, world)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    j0, j1 = int(rowptr[r0]), int(rowptr[r1])
    lrp = (rowptr[r0:r1 + 1] - j0).astype(np.int32)
    return Shard(rank, world, bounds, r0, r1, lrp, colind[j0:j1], val[j0:j1])


def stacked_block(n: int, nnz: int, max_deg: int, rank: int, world: int, seed: int = 1234,
                  gamma: float = 2.3) -> tuple[np.ndarray, np.ndarray]:
    """Row block `rank` of a (world*n)-node power-law graph for weak scaling:
    each rank owns n rows and nnz nonzeros (the per-GPU work of the 1-GPU
    workload), B is replicated with world*n rows, and no collective is on
    the data path. Block r is the Chung-Lu stand-in with seed + r whose
    column c is moved to c*world + ((off[c] + r) % world), off a seeded
    per-column table: monotone in c (rows stay sorted), a hub's copies land
    on different B rows in different blocks, and every block sees the same
    popularity skew as the 1-GPU graph. world = 1 gives the 1-GPU graph
    itself (block 0 = seed)."""
    rp, ci = prep.powerlaw_csr(n, nnz, max_deg, gamma, seed + rank)
    if world == 1:
        return rp, ci
    if world * n > np.iinfo(np.int32).max:
        raise ValueError("stacked_block: world * n exceeds int32 column ids")
    off = np.random.default_rng(seed ^ 0x5EED).integers(0, world, n, dtype=np.int64)
    cj = ci.astype(np.int64)
    cj = cj * world + (off[cj] + rank) % world
    return rp, cj.astype(np.int32)


def gather(local_out, shard: Shard, group=None, compact: bool = True):
    """All-gather the rank slots of a padded [world*max_rows, K] buffer.
    `local_out` must be the padded buffer itself (this rank's rows already in
    its slot); returns the dense [m, K] C if compact, else the buffer."""
    import torch
    import torch.distributed as dist
    mr = shard.max_rows
    K = local_out.shape[1]
    slot = local_out[shard.rank * mr:(shard.rank + 1) * mr]
    dist.all_gather_into_tensor(local_out, slot, group=group)
    if not compact:
        return local_out
    parts = [local_out[r * mr:r * mr + int(shard.bounds[r + 1] - shard.bounds[r])]
             for r in range(shard.world)]
    return torch.cat(parts, 0) if parts else local_out.new_zeros((0, K))


def partitioned_spmm(shard: Shard, B, out, compute: Callable, group=None, compact: bool = True):
    """C = A @ B across ranks: compute(rowptr, colind, val, B, C_slot) fills
    this rank's rows into its slot of `out` ([world*max_rows, K]), then one
    all-gather. `compute` is the HIP op in production (ops.gespmm_csrmm);
    the CPU tests inject the oracle."""
    mr = shard.max_rows
    slot = out[shard.rank * mr:shard.rank * mr + shard.rows]
    compute(shard, B, slot)
    return gather(out, shard, group=group, compact=compact)


def chunk_rows(shard: Shard, nchunks: int) -> int:
    """Rows per chunk (same on every rank: derived from the shared bounds)."""
    return max(1, -(-shard.max_rows // nchunks))


def chunk_range(shard: Shard, rank: int, c: int, nchunks: int) -> tuple[int, int]:
    """Local row range [r0, r1) of rank's chunk c (possibly empty)."""
    cr = chunk_rows(shard, nchunks)
    rows = int(shard.bounds[rank + 1] - shard.bounds[rank])
    r0 = min(c * cr, rows)
    return r0, min(r0 + cr, rows)


def chunked_spmm(shard: Shard, out, compute_chunk: Callable, nchunks: int, group=None,
                 compact: bool = True):
    """C = A @ B across ranks with the all-gather of chunk c overlapping the
    compute of chunk c+1. `out` is [nchunks, world, chunk_rows, K];
    compute_chunk(r0, r1, dest) writes local rows [r0, r1) into dest (a
    [r1-r0, K] view of this rank's slot of chunk c). Returns the dense [m, K]
    C if compact, else `out`."""
    import torch
    import torch.distributed as dist
    nch, world, cr, K = out.shape
    assert nch == nchunks and world == shard.world and cr == chunk_rows(shard, nchunks)
    works = []
    for c in range(nchunks):
        r0, r1 = chunk_range(shard, shard.rank, c, nchunks)
        if r1 > r0:
            compute_chunk(r0, r1, out[c, shard.rank, :r1 - r0])
        works.append(dist.all_gather_into_tensor(out[c].view(world * cr, K),
                                                 out[c, shard.rank], group=group,
                                                 async_op=True))
    for w in works:
        w.wait()
    if not compact:
        return out
    parts = []
    for r in range(world):
        for c in range(nchunks):
            r0, r1 = chunk_range(shard, r, c, nchunks)
            if r1 > r0:
                parts.append(out[c, r, :r1 - r0])
    return torch.cat(parts, 0) if parts else out.new_zeros((0, K))
