"""Row-partitioned multi-GPU SpMM (BASELINE config 4).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).
Every rank holds the full dense B (replicated: 2.5 GB for products at K=256,
far under 288 GB), owns a contiguous nnz-balanced row range of A, computes
its rows of C with the HIP kernel, and the ranks exchange their rows of C
over xGMI. Output rows are independent, and the kernels associate a row's
sum by the row alone (pieces counted from the row's start),
so every rank's rows are bit-identical to the 1-GPU result.

Shards have unequal row counts. C is the caller's contiguous [m, K] matrix
on every rank: the kernel writes this rank's rows in place, and the exchange
(an all-gather with exact, uneven shards) moves every rank's rows straight
into the same rows of every peer's C — no padding, no staging copy, no
compaction after it. xGMI is point-to-point (7 links per GPU), so the exchange
is one batch of isend / irecv pairs, one per peer and direction, all links
busy at once (``exchange_chunk``).

``chunked_spmm`` overlaps the exchange with the compute: each rank's rows are
cut into ``nchunks`` pieces, and piece c's exchange (RCCL on its own stream)
runs while piece c+1 is computed.

``stacked_block`` is the weak-scaling form (bench.py --scaling weak):
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
    rowptr: np.ndarray      # local CSR, rebased to pad = (global offset mod 64)
    colind: np.ndarray      # pad leading filler entries (never read), then the rows'
    val: np.ndarray

    @property
    def rows(self) -> int:
        return self.row1 - self.row0

    @property
    def nnz(self) -> int:
        return int(self.rowptr[-1] - self.rowptr[0])

    @property
    def max_rows(self) -> int:
        return int(np.max(np.diff(self.bounds)))


def make_shard(rowptr: np.ndarray, colind: np.ndarray, val: np.ndarray, rank: int,
               world: int) -> Shard:
    """Cut rank's row range out of a global CSR (host side). The local arrays
    keep every nonzero's array position mod 64 (pad filler entries in front,
    rowptr starting at pad): the K <= 64 lane-group kernel sums a row in
    chains by array position mod its group count, so the shard's rows are
    then bit-identical to the whole matrix's at every K."""
    bounds = prep.partition_rows(rowptr, world)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    j0, j1 = int(rowptr[r0]), int(rowptr[r1])
    pad = j0 % 64
    lrp = (rowptr[r0:r1 + 1] - (j0 - pad)).astype(np.int32)
    lci = np.concatenate([np.zeros(pad, colind.dtype), colind[j0:j1]])
    lv = np.concatenate([np.zeros(pad, val.dtype), val[j0:j1]])
    return Shard(rank, world, bounds, r0, r1, lrp, lci, lv)


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


def chunk_rows(shard: Shard, nchunks: int) -> int:
    """Rows per chunk (same on every rank: derived from the shared bounds)."""
    return max(1, -(-shard.max_rows // nchunks))


def chunk_range(shard: Shard, rank: int, c: int, nchunks: int) -> tuple[int, int]:
    """Local row range [r0, r1) of rank's chunk c (possibly empty)."""
    cr = chunk_rows(shard, nchunks)
    rows = int(shard.bounds[rank + 1] - shard.bounds[rank])
    r0 = min(c * cr, rows)
    return r0, min(r0 + cr, rows)


def _rows_of(C, shard: Shard, rank: int, c: int, nchunks: int):
    """The global rows of rank's chunk c as a contiguous view of C (None if
    the chunk is empty)."""
    r0, r1 = chunk_range(shard, rank, c, nchunks)
    if r1 <= r0:
        return None
    g0 = int(shard.bounds[rank])
    return C[g0 + r0:g0 + r1]


def exchange_chunk(C, shard: Shard, c: int, nchunks: int, group=None) -> list:
    """Start the exchange of chunk c: this rank's chunk-c rows go to every peer
    and every peer's chunk-c rows land in place in C (an all-gather with
    uneven, exact shards). xGMI is point-to-point, so each rank sends its
    rows straight to each peer over that peer's link and receives the peers'
    rows the same way: one batch of isend / irecv pairs (one ncclGroup on
    RCCL), every link busy at once. Both sides derive the chunk ranges from
    the shared bounds, so an empty chunk is skipped on both. Returns the
    requests (empty at world 1: nothing to move)."""
    import torch.distributed as dist
    ops = []
    mine = _rows_of(C, shard, shard.rank, c, nchunks)
    for q in range(shard.world):
        if q == shard.rank:
            continue
        if mine is not None:
            ops.append(dist.P2POp(dist.isend, mine, q, group=group))
        theirs = _rows_of(C, shard, q, c, nchunks)
        if theirs is not None:
            ops.append(dist.P2POp(dist.irecv, theirs, q, group=group))
    return dist.batch_isend_irecv(ops) if ops else []


def _check_out(C, shard: Shard) -> None:
    m = int(shard.bounds[-1])
    if C.dim() != 2 or C.shape[0] != m or not C.is_contiguous():
        raise ValueError(f"C must be the contiguous [{m}, K] output, got {tuple(C.shape)}")


def gather(C, shard: Shard, group=None):
    """Complete C on every rank: this rank's rows [row0, row1) are already in
    place; the other ranks' rows arrive in place (exchange_chunk, one chunk).
    Returns C."""
    _check_out(C, shard)
    for w in exchange_chunk(C, shard, 0, 1, group):
        w.wait()
    return C


def partitioned_spmm(shard: Shard, B, C, compute: Callable, group=None):
    """C = A @ B across ranks: compute(shard, B, rows) fills this rank's rows
    (a [rows, K] view of the [m, K] C), then the exchange. `compute` is the
    HIP op in production (ops.csrmm); the CPU tests inject the oracle."""
    _check_out(C, shard)
    compute(shard, B, C[shard.row0:shard.row1])
    return gather(C, shard, group=group)


def chunked_spmm(shard: Shard, C, compute_chunk: Callable, nchunks: int, group=None):
    """C = A @ B across ranks with the exchange of chunk c overlapping the
    compute of chunk c+1. C is the contiguous [m, K] output on every rank;
    compute_chunk(r0, r1, dest) writes local rows [r0, r1) into dest (their
    [r1-r0, K] view of C). Returns C, complete on every rank."""
    _check_out(C, shard)
    works = []
    for c in range(nchunks):
        dest = _rows_of(C, shard, shard.rank, c, nchunks)
        if dest is not None:
            r0, r1 = chunk_range(shard, shard.rank, c, nchunks)
            compute_chunk(r0, r1, dest)
        works += exchange_chunk(C, shard, c, nchunks, group)
    for w in works:
        w.wait()
    return C
