"""The CSR kernels' grid-independent association, on the CPU:

* the piece-cut model of csr_kernels.hip (snap_cut, wave_range, the split-row
  keys and ticket counts) restated in Python: for random power-law matrices and
  many grid sizes, every piece of every row lies inside one wave's range, the
  ranges tile the merge path, split rows have distinct keys, and the pieces
  their waves store add up to the row's piece count — so the last arrival is
  well defined and no slot is written twice;
* the oracle's piece sum (oracle_csrmm_pieces_f32) is the sequential chain of
  oracle_csrmm_f32 for rows of at most 128 nonzeros, and within the fp32 bar of
  the f64 product for longer ones.
The GPU tests (test_gpu_csr.py) then hold the kernels to the piece oracle bit
for bit."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import (TOL_F32, assert_normwise, oracle_csrmm_f32, oracle_csrmm_f64,
                     oracle_csrmm_pieces_f32)

PIECE_MIN, MAX_PIECES = 128, 64


def piece_len(L: int) -> int:
    return max(PIECE_MIN, (L + MAX_PIECES - 1) // MAX_PIECES)


def merge_point(rp: np.ndarray, d: int) -> tuple[int, int]:
    """(i, j) on the merge path at diagonal d (csr_kernels.hip merge_search2):
    i = the number of rows whose end step, at diagonal (r + 1) + rowptr[r + 1],
    lies at or before d; j = d - i."""
    m = rp.size - 1
    lo, hi = max(0, d - int(rp[-1])), min(d, m)
    while lo < hi:  # first i in [lo, hi) whose end is not consumed at d
        mid = (lo + hi) // 2
        if int(rp[mid + 1]) <= d - mid - 1:
            lo = mid + 1
        else:
            hi = mid
    return lo, d - lo


def snap(rp: np.ndarray, i: int, j: int) -> tuple[int, int]:
    m = rp.size - 1
    if i >= m:
        return i, j
    rs, re = int(rp[i]), int(rp[i + 1])
    if j <= rs:
        return i, j
    if j >= re:
        return i + 1, re
    T = piece_len(re - rs)
    return i, rs + (j - rs) // T * T


def wave_pieces(rp: np.ndarray, nwaves: int):
    """Per wave: its snapped range and the (row, piece) pairs it sums."""
    m, nnz = rp.size - 1, int(rp[-1])
    total = m + nnz
    per = -(-total // nwaves)
    out = []
    for w in range(nwaves):
        d0, d1 = min(w * per, total), min(w * per + per, total)
        i0, j0 = snap(rp, *merge_point(rp, d0))
        i1, j1 = snap(rp, *merge_point(rp, d1))
        pieces = []
        for r in range(i0, min(i1 + 1, m)):
            rs, re = int(rp[r]), int(rp[r + 1])
            lo, hi = max(rs, j0), min(re, j1)
            T = piece_len(re - rs)
            for k in range((re - rs + T - 1) // T):
                a, b = rs + k * T, min(rs + (k + 1) * T, re)
                if a < hi and b > lo:
                    assert lo <= a and b <= hi, f"wave {w} cuts piece {k} of row {r}"
                    pieces.append((r, k))
        out.append(((i0, j0), (i1, j1), per, pieces))
    return out


@pytest.mark.parametrize("seed,m,deg_hi,hubs", [(1, 3000, 6, 4000), (2, 500, 40, 20000),
                                                (3, 2000, 3, 300), (4, 50, 0, 9000)])
@pytest.mark.parametrize("nwaves", [1, 2, 7, 64, 333, 1024])
def test_every_piece_in_one_wave(seed, m, deg_hi, hubs, nwaves):
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, deg_hi + 1, m)
    deg[rng.random(m) < 0.2] = 0
    for r in rng.choice(m, 3, replace=False):
        deg[r] = hubs
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    waves = wave_pieces(rp, nwaves)
    # the ranges tile the path in order
    prev = (0, 0)
    for (a, b, _, _) in waves:
        assert a == prev or (a[0] + a[1]) >= (prev[0] + prev[1])
        assert (b[0] + b[1]) >= (a[0] + a[1])
        prev = b
    assert prev == (m, int(rp[-1]))
    # every piece of every row summed exactly once
    seen = {}
    for w, (_, _, _, pieces) in enumerate(waves):
        for p in pieces:
            assert p not in seen, f"piece {p} in waves {seen[p]} and {w}"
            seen[p] = w
    for r in range(m):
        L = int(rp[r + 1] - rp[r])
        npc = -(-L // piece_len(L))
        assert all((r, k) in seen for k in range(npc))
    # split rows: keys (r + rs) // per distinct, stored counts add up to np
    per = waves[0][2]
    owners = {}
    for (r, k), w in seen.items():
        owners.setdefault(r, set()).add(w)
    keys = {}
    for r, ws in owners.items():
        if len(ws) > 1:
            key = (r + int(rp[r])) // per
            assert key not in keys, f"rows {keys[key]} and {r} share key {key}"
            keys[key] = r
            assert key < nwaves


def test_piece_oracle_is_the_sequential_chain_for_short_rows(oracle):
    rng = np.random.default_rng(9)
    m, k, K = 400, 3000, 16
    deg = rng.integers(0, 129, m)
    deg[::37] = rng.integers(129, 2500, deg[::37].size)  # a few multi-piece rows
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = rng.integers(0, k, int(rp[-1])).astype(np.int32)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    B = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    seq = oracle_csrmm_f32(oracle, m, K, rp, ci, v, B, K, 0).reshape(m, K)
    pcs = oracle_csrmm_pieces_f32(oracle, m, K, rp, ci, v, B, K, 0).reshape(m, K)
    short = deg <= 128
    assert np.array_equal(seq[short], pcs[short])
    assert not np.array_equal(seq[~short], pcs[~short])  # other association, same bar
    ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, B, K, 0)
    assert_normwise(pcs, ref, absd, TOL_F32, "piece sums")
    assert [oracle.oracle_csr_piece_len(L) for L in (0, 128, 129, 2048, 2049, 17481)] == \
        [piece_len(L) for L in (0, 128, 129, 2048, 2049, 17481)]


def test_piece_oracle_epilogue(oracle):
    """alpha / beta and both storage orders go through the same epilogue as
    the sequential oracle: fma(beta, C, alpha * x)."""
    rng = np.random.default_rng(10)
    m, k, K = 120, 200, 8
    deg = rng.integers(0, 300, m)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = rng.integers(0, k, int(rp[-1])).astype(np.int32)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    B = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    x = oracle_csrmm_pieces_f32(oracle, m, K, rp, ci, v, B, K, 0).reshape(m, K)
    got = oracle_csrmm_pieces_f32(oracle, m, K, rp, ci, v, np.ascontiguousarray(B.T), k, 1,
                                  alpha=0.7, beta=-1.3, C=np.ascontiguousarray(C0.T), ldc=m,
                                  order_c=1).reshape(K, m).T
    # fma(beta, C0, alpha * x): one rounding of the exact f64 sum (numpy has no fma)
    want = np.float64(np.float32(-1.3)) * C0 + (np.float32(0.7) * x).astype(np.float64)
    assert np.allclose(got, want, rtol=1e-6, atol=1e-7)
