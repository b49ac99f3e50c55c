"""Shared test helpers: oracle loading (tests only), golden fixtures,
tolerance checks."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

P = ctypes.c_void_p
I, I64, F, D, U64 = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_uint64

# Norm-wise relative tolerance for fp32 SpMM (north_star: 1e-5 relative):
# |C - C_ref| <= TOL_F32 * sum_j |a_j * b_j| + tiny, per element.
TOL_F32 = 1e-5
# fp16 inputs with fp32 accumulation, checked against the exact (float64)
# product of the SAME fp16 values.
TOL_F16_ACC = 1e-5


def _build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)


def load_oracle() -> ctypes.CDLL:
    if not os.path.exists(ORACLE_SO):
        _build_oracle()
    L = ctypes.CDLL(ORACLE_SO)
    sig = {
        "oracle_rng_seed": (None, [U64]),
        "oracle_random_array": (None, [I64, F, F, P]),
        "oracle_random_csr": (I64, [I, I, F, F, F, P, P, P, I64]),
        "oracle_csrmm_f32": (None, [I, I, P, P, P, I, P, I, I, F, F, P, I, I]),
        "oracle_csrmm_pieces_f32": (None, [I, I, P, P, P, I, P, I, I, F, F, P, I, I]),
        "oracle_csr_piece_len": (I, [I]),
        "oracle_csrmm_f64": (None, [I, I, P, P, P, I, P, I, I, P, P]),
        "oracle_csrmm_d": (None, [I, I, P, P, P, I, P, I, I, ctypes.c_double, ctypes.c_double,
                                  P, I, I]),
        "oracle_bsrmm_d": (None, [I, I, I, I, P, P, P, P, I, I, ctypes.c_double,
                                  ctypes.c_double, P, I, I]),
        "oracle_spmm_cc_csr": (None, [I64, I64, P, P, P, I64, P]),
        "oracle_spmm_cc_coo": (None, [I64, I64, I64, P, P, P, I64, P]),
        "oracle_coo2csr": (None, [P, I, I, I, P]),
        "oracle_num_threads": (I, []),
        "oracle_reorder": (I, [I, I, P, P, P, P, P]),
        "oracle_bsrmm_f32": (None, [I, I, I, I, P, P, P, P, I, I, F, F, P, I, I]),
        "oracle_bsrmm_f64": (None, [I, I, I, I, P, P, P, P, I, I, I, P, P]),
        "oracle_csr2bsr_nnz": (I64, [I, I, P, P, P]),
        "oracle_csr2bsr": (None, [I, I, I, P, P, P, P, P, P]),
        "oracle_bsr2csr": (None, [I, I, I, P, P, P, P, P, P]),
        "oracle_divide": (I, [I, I, F, P, P, P, P, P, P, P, P, P, I64, P]),
    }
    for k, (r, a) in sig.items():
        f = getattr(L, k)
        f.restype = r
        f.argtypes = a
    return L


def ptr(a: np.ndarray | None):
    return ctypes.c_void_p(a.ctypes.data if a is not None and a.size else 0)


def load_golden() -> dict:
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        kats = json.load(f)
    with open(os.path.join(GOLDEN, "ref_config1.json")) as f:
        cfg1 = json.load(f)
    npz = np.load(os.path.join(GOLDEN, "ref_host.npz"), allow_pickle=False)
    return {"kats": kats, "config1": cfg1, "ref": {k: npz[k] for k in npz.files}}


# ------------------------------------------------------------ oracle calls
def oracle_csrmm_f32(L, m, n, rowptr, colind, val, B, ldb, order_b, alpha=1.0, beta=0.0,
                     C=None, ldc=None, order_c=0, base=0):
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    if ldc is None:
        ldc = n if order_c == 0 else m
    if C is None:
        C = np.zeros(m * ldc if order_c == 0 else n * ldc, np.float32)
    C = np.ascontiguousarray(C, np.float32).copy()
    L.oracle_csrmm_f32(m, n, ptr(rowptr), ptr(colind), ptr(val), base, ptr(B), ldb, order_b,
                       alpha, beta, ptr(C), ldc, order_c)
    return C


def oracle_csrmm_pieces_f32(L, m, n, rowptr, colind, val, B, ldb, order_b, alpha=1.0,
                            beta=0.0, C=None, ldc=None, order_c=0, base=0):
    """The HIP CSR kernels' association: sequential fp32 FMA
    chains over pieces of max(128, ceil(L / 64)) nonzeros from each row's start,
    added left to right; the main kernel matches it bit for bit at any grid."""
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    if ldc is None:
        ldc = n if order_c == 0 else m
    if C is None:
        C = np.zeros(m * ldc if order_c == 0 else n * ldc, np.float32)
    C = np.ascontiguousarray(C, np.float32).copy()
    L.oracle_csrmm_pieces_f32(m, n, ptr(rowptr), ptr(colind), ptr(val), base, ptr(B), ldb,
                              order_b, alpha, beta, ptr(C), ldc, order_c)
    return C


def oracle_csrmm_d(L, m, n, rowptr, colind, val, B, ldb, order_b, alpha=1.0, beta=0.0,
                   C=None, ldc=None, order_c=0, base=0):
    """gespmm_csrmm<double> semantics: sequential fp64 FMA in CSR order."""
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    val = np.ascontiguousarray(val, np.float64)
    B = np.ascontiguousarray(B, np.float64)
    if ldc is None:
        ldc = n if order_c == 0 else m
    if C is None:
        C = np.zeros(m * ldc if order_c == 0 else n * ldc, np.float64)
    C = np.ascontiguousarray(C, np.float64).copy()
    L.oracle_csrmm_d(m, n, ptr(rowptr), ptr(colind), ptr(val), base, ptr(B), ldb, order_b,
                     alpha, beta, ptr(C), ldc, order_c)
    return C


def oracle_bsrmm_d(L, direction, mb, n, bs, rowptr, colind, val, B, ldb, order_b, alpha=1.0,
                   beta=0.0, C=None, ldc=None, order_c=0):
    """rocsparse_bsrmm_template<double> semantics: blocks in order, q = 0..bs-1."""
    m = mb * bs
    if ldc is None:
        ldc = n if order_c == 0 else m
    if C is None:
        C = np.zeros(m * ldc if order_c == 0 else n * ldc, np.float64)
    C = np.ascontiguousarray(C, np.float64).copy()
    args = [np.ascontiguousarray(a, t) for a, t in
            ((rowptr, np.int32), (colind, np.int32), (val, np.float64), (B, np.float64))]
    L.oracle_bsrmm_d(direction, mb, n, bs, *[ptr(a) for a in args], ldb, order_b, alpha, beta,
                     ptr(C), ldc, order_c)
    return C


def oracle_csrmm_f64(L, m, n, rowptr, colind, val, B, ldb, order_b, base=0):
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    C = np.zeros((m, n), np.float64)
    A = np.zeros((m, n), np.float64)
    L.oracle_csrmm_f64(m, n, ptr(rowptr), ptr(colind), ptr(val), base, ptr(B), ldb, order_b,
                       ptr(C), ptr(A))
    return C, A


def oracle_bsrmm_f32(L, direction, mb, n, bs, rowptr, colind, val, B, ldb, order_b, alpha=1.0,
                     beta=0.0, C=None, ldc=None, order_c=0):
    m = mb * bs
    if ldc is None:
        ldc = n if order_c == 0 else m
    if C is None:
        C = np.zeros(m * ldc if order_c == 0 else n * ldc, np.float32)
    C = np.ascontiguousarray(C, np.float32).copy()
    args = [np.ascontiguousarray(a, t) for a, t in
            ((rowptr, np.int32), (colind, np.int32), (val, np.float32), (B, np.float32))]
    L.oracle_bsrmm_f32(direction, mb, n, bs, *[ptr(a) for a in args], ldb, order_b, alpha, beta,
                       ptr(C), ldc, order_c)
    return C


def oracle_bsrmm_f64(L, direction, mb, n, bs, rowptr, colind, val, B, ldb, order_b, half=False):
    m = mb * bs
    C = np.zeros((m, n), np.float64)
    A = np.zeros((m, n), np.float64)
    vt = np.float16 if half else np.float32
    args = [np.ascontiguousarray(rowptr, np.int32), np.ascontiguousarray(colind, np.int32),
            np.ascontiguousarray(val, vt), np.ascontiguousarray(B, vt)]
    L.oracle_bsrmm_f64(direction, mb, n, bs, *[ptr(a) for a in args], ldb, order_b, int(half),
                       ptr(C), ptr(A))
    return C, A


def oracle_divide(L, n, bs, density, rowptr, colind, val):
    """divide_matrix with values -> (csr_rp, csr_ci, csr_v, bsr_rp, bsr_ci, bsr_v)."""
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    nb = (n + bs - 1) // bs
    cap = nb * nb if density <= 0 else max(colind.size, 1)
    crp, cci, cv = (np.zeros(n + 1, np.int32), np.zeros(max(colind.size, 1), np.int32),
                    np.zeros(max(colind.size, 1), np.float32))
    brp, bci, bv = np.zeros(nb + 1, np.int32), np.zeros(cap, np.int32), \
        np.zeros(cap * bs * bs, np.float32)
    out = np.zeros(2, np.int64)
    assert L.oracle_divide(n, bs, density, ptr(rowptr), ptr(colind), ptr(val), ptr(crp),
                           ptr(cci), ptr(cv), ptr(brp), ptr(bci), ptr(bv), cap, ptr(out)) == 0
    c, b = int(out[0]), int(out[1])
    return crp, cci[:c].copy(), cv[:c].copy(), brp, bci[:b].copy(), bv[:b * bs * bs].copy()


def assert_normwise(got, ref64, absdot, tol, what=""):
    """|got - ref| <= tol * absdot + 1e-30 elementwise (float64 comparison)."""
    got = np.asarray(got, np.float64)
    err = np.abs(got - ref64)
    bound = tol * absdot + 1e-30
    bad = err > bound
    if bad.any():
        i = np.argmax(err - bound)
        raise AssertionError(
            f"{what}: {int(bad.sum())} / {bad.size} elements outside the norm-wise tolerance "
            f"{tol}; worst flat index {i}: got {got.flat[i]!r} ref {ref64.flat[i]!r} "
            f"|a||b| {absdot.flat[i]!r}")


def oracle_reorder(L, kind: str, rowptr, colind, perm=None):
    """Reordered CSR from the oracle's restatement of reorder_strategy.cc."""
    k = {"degree": 0, "bfs": 1, "rcm": 2, "permute": 3}[kind]
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    colind = np.ascontiguousarray(colind, np.int32)
    n = rowptr.size - 1
    perm = np.zeros(max(n, 1), np.int32) if perm is None else np.ascontiguousarray(perm, np.int32)
    orp, oci = np.zeros(n + 1, np.int32), np.zeros(max(colind.size, 1), np.int32)
    assert L.oracle_reorder(k, n, ptr(rowptr), ptr(colind), ptr(perm), ptr(orp), ptr(oci)) == 0
    return orp, oci[:colind.size]


def load_reorder_golden():
    return np.load(os.path.join(GOLDEN, "ref_reorder.npz"), allow_pickle=False)
