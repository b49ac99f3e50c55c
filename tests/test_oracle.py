"""The oracle pinned against the reference: its KAT programs, its RNG stream,
its csr2bsr / calculateNnzb index arrays (golden fixtures generated from the
reference's own host code), and — where the reference tree is present — the
reference code itself, live. CPU only."""
from __future__ import annotations

import ctypes
import hashlib
import os

import numpy as np
import pytest

from helpers import (REF_SO, oracle_bsrmm_d, oracle_bsrmm_f32, oracle_csrmm_d, oracle_csrmm_f32,
                     ptr)


def test_rng_stream_matches_reference(oracle, golden):
    # load_data.cc:12,29-40 — randomDenseMatrix(64, 64) from a fresh generator.
    oracle.oracle_rng_seed(1234)
    a = np.empty(64 * 64, np.float32)
    oracle.oracle_random_array(a.size, -1.0, 1.0, ptr(a))
    assert np.array_equal(a, golden["ref"]["dense_64x64"])
    # SURVEY.md §4 fingerprint of randomDenseMatrix(2, 4).
    np.testing.assert_allclose(a[:8], [0.894463181, -0.895553231, 0.948636532, 0.891496778,
                                       -0.628704309, 0.897466779, 0.765075207, 0.888155222],
                               rtol=0, atol=5e-9)


@pytest.mark.parametrize("shape", [(64, 80, 0.1), (300, 257, 0.03), (1000, 1200, 0.01)])
def test_random_csr_matches_reference(oracle, golden, shape):
    m, n, p = shape
    oracle.oracle_rng_seed(1234)
    cap = int(m * n * p * 1.5) + 1024
    rp, ci, v = np.zeros(m + 1, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.float32)
    nnz = oracle.oracle_random_csr(m, n, p, -1.0, 1.0, ptr(rp), ptr(ci), ptr(v), cap)
    key = f"csr_{m}_{n}_{p}"
    assert np.array_equal(rp, golden["ref"][key + "_rowptr"])
    assert np.array_equal(ci[:nnz], golden["ref"][key + "_colind"])
    assert np.array_equal(v[:nnz], golden["ref"][key + "_val"])


def test_config1_digest(oracle, golden):
    """BASELINE configs[0]: randomCSRMatrix(16384, 16384, 2^-10) then
    randomDenseMatrix(16384, 32) — digests of the reference's own output."""
    c = golden["config1"]
    m = c["m"]
    oracle.oracle_rng_seed(1234)
    cap = 400000
    rp, ci, v = np.zeros(m + 1, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.float32)
    nnz = oracle.oracle_random_csr(m, m, c["p"], -1.0, 1.0, ptr(rp), ptr(ci), ptr(v), cap)
    B = np.empty(m * c["K"], np.float32)
    oracle.oracle_random_array(B.size, -1.0, 1.0, ptr(B))
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert nnz == c["nnz"]
    assert sha(rp) == c["rowptr_sha256"]
    assert sha(ci[:nnz]) == c["colind_sha256"]
    assert sha(v[:nnz]) == c["val_sha256"]
    assert sha(B) == c["B_sha256"]


def test_kat_csrmm_cu(oracle, golden):
    k = golden["kats"]["csrmm_cu"]
    C = oracle_csrmm_f32(oracle, k["m"], k["n"], k["rowptr"], k["colind"], k["val"],
                         np.array(k["B_colmajor"], np.float32), k["ldb"], 1, ldc=k["ldc"],
                         order_c=1)
    assert C.tolist() == k["C_colmajor"] == k["survey"]


def test_kat_try_cublas_cu(oracle, golden):
    k = golden["kats"]["try_cublas_cu"]
    C = oracle_csrmm_f32(oracle, k["m"], k["n"], k["rowptr"], k["colind"], k["val"],
                         np.array(k["B_colmajor"], np.float32), k["ldb"], 1, ldc=k["ldc"],
                         order_c=1)
    assert C.tolist() == k["C_colmajor"]


def test_kat_bsrmm_cu(oracle, golden):
    k = golden["kats"]["bsrmm_cu"]
    C = oracle_bsrmm_f32(oracle, k["dir"], k["mb"], k["n"], k["bs"], k["rowptr"], k["colind"],
                         k["val"], np.array(k["B_colmajor"], np.float32), k["ldb"], 1,
                         ldc=k["ldc"], order_c=1)
    assert C.tolist() == k["C_colmajor"]


def test_kat_block_cublas_cu(oracle, golden):
    k = golden["kats"]["block_cublas_cu"]
    C = oracle_bsrmm_f32(oracle, k["dir"], k["mb"], k["n"], k["bs"], k["rowptr"], k["colind"],
                         k["val"], np.array(k["B_rowmajor"], np.float32), k["ldb"], 0,
                         beta=k["beta"], C=np.zeros(12, np.float32), ldc=k["ldc"], order_c=1)
    assert C.tolist() == k["C_colmajor"]


def test_kat_fp64_forms(oracle, golden):
    """T = double (gespmm_csrmm<T>, rocsparse_bsrmm_template<T>): the KAT
    programs' integer-valued operands give the same answers in fp64."""
    k = golden["kats"]["csrmm_cu"]
    C = oracle_csrmm_d(oracle, k["m"], k["n"], k["rowptr"], k["colind"], k["val"],
                       np.array(k["B_colmajor"], np.float64), k["ldb"], 1, ldc=k["ldc"],
                       order_c=1)
    assert C.tolist() == k["C_colmajor"]
    k = golden["kats"]["bsrmm_cu"]
    C = oracle_bsrmm_d(oracle, k["dir"], k["mb"], k["n"], k["bs"], k["rowptr"], k["colind"],
                       k["val"], np.array(k["B_colmajor"], np.float64), k["ldb"], 1,
                       ldc=k["ldc"], order_c=1)
    assert C.tolist() == k["C_colmajor"]


@pytest.mark.parametrize("bs,direction", [(1, 0), (3, 1), (8, 0)])
def test_fp64_oracles_vs_dense(oracle, bs, direction):
    """fp64 oracles against a dense numpy product (alpha/beta epilogue too)."""
    rng = np.random.default_rng(5)
    mb, kb, n = 13, 11, 7
    mask = rng.random((mb, kb)) < 0.3
    brp = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
    bci = np.nonzero(mask)[1].astype(np.int32)
    blocks = rng.standard_normal((bci.size, bs, bs))
    A = np.zeros((mb * bs, kb * bs))
    for r in range(mb):
        for k in range(brp[r], brp[r + 1]):
            A[r * bs:(r + 1) * bs, bci[k] * bs:(bci[k] + 1) * bs] = blocks[k]
    vals = blocks if direction == 0 else blocks.transpose(0, 2, 1)
    B = rng.standard_normal((kb * bs, n))
    C0 = rng.standard_normal((mb * bs, n))
    got = oracle_bsrmm_d(oracle, direction, mb, n, bs, brp, bci, vals.ravel(), B, n, 0,
                         alpha=0.5, beta=2.0, C=C0.ravel()).reshape(mb * bs, n)
    np.testing.assert_allclose(got, 0.5 * A @ B + 2.0 * C0, rtol=1e-12, atol=1e-12)
    rows, cols = np.nonzero(A)
    rp = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=A.shape[0]))])
    got = oracle_csrmm_d(oracle, A.shape[0], n, rp, cols, A[rows, cols], B, n, 0)
    np.testing.assert_allclose(got.reshape(-1, n), A @ B, rtol=1e-12, atol=1e-12)


def test_kat_spmm_cc_small(oracle, golden):
    k = golden["kats"]["spmm_cc_small"]
    ip = np.array(k["indptr"], np.int64)
    ix = np.array(k["indices"], np.int64)
    D = np.array(k["dense"], np.float64)
    out = np.zeros(k["m"] * k["n"], np.float64)
    oracle.oracle_spmm_cc_csr(k["m"], k["n"], ptr(ip), ptr(ix), ptr(D), k["n"], ptr(out))
    assert out.tolist() == k["out"]


def test_kat_spmm_cc_small_coo(oracle, golden):
    """spmm.cc:54-61 test_small_coo_spmm: the same product from COO rows
    {0, 1, 1}, cols {1, 0, 2} (spmm.cc:56) through coo_spmm (:27-43)."""
    k = golden["kats"]["spmm_cc_small"]
    row = np.array([0, 1, 1], np.int64)
    col = np.array([1, 0, 2], np.int64)
    D = np.array(k["dense"], np.float64)
    out = np.full(k["m"] * k["n"], np.nan)
    oracle.oracle_spmm_cc_coo(k["m"], k["n"], 3, ptr(row), ptr(col), ptr(D), k["n"], ptr(out))
    assert out.tolist() == k["out"]


def test_coo_spmm_matches_csr_spmm(oracle):
    """coo_spmm and csr_spmm of spmm.cc on one random pattern (double, unit
    values; the atomic adds may reorder a sum, hence the 1e-12 bar)."""
    from spmm_hip import prep
    prep.rng_seed(1234)
    rp, ci, _ = prep.random_csr(3000, 2500, 0.01)
    m, K = 3000, 17
    D = np.random.default_rng(3).uniform(-1, 1, (2500, K))
    row = np.repeat(np.arange(m, dtype=np.int64), np.diff(rp))
    col = ci.astype(np.int64)
    a, b = np.empty((m, K)), np.empty((m, K))
    ip = rp.astype(np.int64)
    oracle.oracle_spmm_cc_csr(m, K, ptr(ip), ptr(col), ptr(D), K, ptr(a))
    oracle.oracle_spmm_cc_coo(m, K, col.size, ptr(row), ptr(col), ptr(D), K, ptr(b))
    assert np.abs(a - b).max() <= 1e-12


def test_coo2csr_kat(oracle, golden):
    """cusparseXcoo2csr on csrmm.cu's COO (csrmm.cu:47-99,148-149) gives the
    KAT's row pointer, in both index bases; empty rows and trailing rows too."""
    k = golden["kats"]["csrmm_cu"]
    rows = np.array(k["coo_row"], np.int32)
    for base in (0, 1):
        out = np.zeros(k["m"] + 1, np.int32)
        rb = rows + base
        oracle.oracle_coo2csr(ptr(rb), rows.size, k["m"], base, ptr(out))
        assert (out - base).tolist() == k["rowptr"]
    rows = np.array([1, 1, 4, 4, 4], np.int32)  # rows 0, 2, 3, 5, 6 empty
    out = np.zeros(8, np.int32)
    oracle.oracle_coo2csr(ptr(rows), 5, 7, 0, ptr(out))
    assert out.tolist() == [0, 0, 2, 2, 2, 5, 5, 5]


def _divide_fixture(golden, g, bs, tag="all"):
    r = golden["ref"]
    return [r[f"{g}_bs{bs}_{tag}_{nm}"] for nm in ("csr_rp", "csr_ci", "bsr_rp", "bsr_ci",
                                                    "bsr_val")]


@pytest.mark.parametrize("g", ["rand300", "band200"])
@pytest.mark.parametrize("bs", [2, 4, 16, 32])
def test_csr2bsr_matches_divide_matrix(oracle, golden, g, bs):
    """divide_matrix at density 1e-9 keeps every nonempty block: its BSR part
    is csr2bsr(DIRECTION_ROW) of the unit-valued pattern (divide.cu:52-127)."""
    rp, ci = golden["ref"][f"{g}_rowptr"], golden["ref"][f"{g}_colind"]
    n = rp.size - 1
    _, csr_ci, brp_ref, bci_ref, bval_ref = _divide_fixture(golden, g, bs)
    assert csr_ci.size == 0  # nothing left in the CSR remainder
    mb = (n + bs - 1) // bs
    brp = np.zeros(mb + 1, np.int32)
    nnzb = oracle.oracle_csr2bsr_nnz(n, bs, ptr(rp), ptr(ci), ptr(brp))
    assert nnzb == golden["ref"][f"{g}_bs{bs}_nnzb"][0]  # calculateNnzb
    bci = np.zeros(nnzb, np.int32)
    bval = np.zeros(nnzb * bs * bs, np.float32)
    ones = np.ones(ci.size, np.float32)
    oracle.oracle_csr2bsr(0, n, bs, ptr(rp), ptr(ci), ptr(ones), ptr(brp), ptr(bci), ptr(bval))
    assert np.array_equal(brp, brp_ref)
    assert np.array_equal(bci, bci_ref)
    assert np.array_equal(bval, bval_ref)


def test_bsr2csr_roundtrip_preserves_product(oracle, golden):
    """csr2bsr -> bsr2csr keeps every block (explicit zeros, nnz = nnzb*bs^2,
    bsr2csr.cu:177) and the SpMM result (csr2bsr.cu / bsr2csr.cu differential)."""
    rp, ci = golden["ref"]["csr_300_257_0.03_rowptr"], golden["ref"]["csr_300_257_0.03_colind"]
    v = golden["ref"]["csr_300_257_0.03_val"]
    m, bs, K = 300, 4, 7
    mb = (m + bs - 1) // bs
    brp = np.zeros(mb + 1, np.int32)
    nnzb = oracle.oracle_csr2bsr_nnz(m, bs, ptr(rp), ptr(ci), ptr(brp))
    bci, bval = np.zeros(nnzb, np.int32), np.zeros(nnzb * bs * bs, np.float32)
    for d in (0, 1):
        oracle.oracle_csr2bsr(d, m, bs, ptr(rp), ptr(ci), ptr(v), ptr(brp), ptr(bci), ptr(bval))
        rp2 = np.zeros(mb * bs + 1, np.int32)
        ci2 = np.zeros(nnzb * bs * bs, np.int32)
        v2 = np.zeros(nnzb * bs * bs, np.float32)
        oracle.oracle_bsr2csr(d, mb, bs, ptr(brp), ptr(bci), ptr(bval), ptr(rp2), ptr(ci2),
                              ptr(v2))
        assert rp2[-1] == nnzb * bs * bs
        rng = np.random.default_rng(0)
        B = rng.uniform(-1, 1, (mb * bs + 8) * K).astype(np.float32)  # rows >= nb*bs
        c1 = oracle_csrmm_f32(oracle, m, K, rp, ci, v, B, K, 0)
        c2 = oracle_csrmm_f32(oracle, mb * bs, K, rp2, ci2, v2, B, K, 0)[: m * K]
        c3 = oracle_bsrmm_f32(oracle, d, mb, K, bs, brp, bci, bval, B, K, 0)[: m * K]
        np.testing.assert_allclose(c2, c1, rtol=0, atol=1e-5)
        np.testing.assert_allclose(c3, c1, rtol=0, atol=1e-5)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference tree / oracle/_ref not built")
def test_live_reference_divide_matrix_random(oracle):
    """Live cross-check against the reference's divide_matrix on fresh inputs."""
    L = ctypes.CDLL(REF_SO)
    L.ref_divide_matrix.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    L.ref_divide_fetch.argtypes = [ctypes.c_void_p] * 5
    rng = np.random.default_rng(7)
    for trial in range(5):
        n = int(rng.integers(1, 400))
        deg = rng.integers(0, 12, n)
        rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
        ci = np.concatenate([np.sort(rng.choice(n, min(d, n), replace=False))
                             for d in deg]).astype(np.int32) if rp[-1] else np.zeros(0, np.int32)
        for bs in (3, 8, 32):
            sizes = np.zeros(5, np.int64)
            L.ref_divide_matrix(n, ptr(rp), ptr(ci), bs, 1e-9, ptr(sizes))
            arrs = [np.zeros(int(s), t) for s, t in
                    zip(sizes, [np.int32, np.int32, np.int32, np.int32, np.float32])]
            L.ref_divide_fetch(*[ptr(a) for a in arrs])
            mb = (n + bs - 1) // bs
            brp = np.zeros(mb + 1, np.int32)
            nnzb = oracle.oracle_csr2bsr_nnz(n, bs, ptr(rp), ptr(ci), ptr(brp))
            bci, bval = np.zeros(nnzb, np.int32), np.zeros(nnzb * bs * bs, np.float32)
            ones = np.ones(max(ci.size, 1), np.float32)  # keep alive across the call
            oracle.oracle_csr2bsr(0, n, bs, ptr(rp), ptr(ci), ptr(ones), ptr(brp), ptr(bci),
                                  ptr(bval))
            assert np.array_equal(brp, arrs[2]) and np.array_equal(bci, arrs[3])
            assert np.array_equal(bval, arrs[4])
