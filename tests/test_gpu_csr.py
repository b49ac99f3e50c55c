"""Path A parity on the GPU: CSR x dense through the C ABI vs the oracle.

Bar (north_star): within 1e-5 norm-wise relative of the reference semantics
(sequential fp32 FMA in CSR order, gespmm_csrmm.h:124-129). Beyond the bar the
main kernel is bit-identical to the piece oracle (oracle_csrmm_pieces_f32,
DESIGN.md §3c) at every grid, and so to the sequential oracle on every row of
at most 128 nonzeros; the K <= 64 lane-group kernel gives the same bits at
every grid and shard."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from helpers import (TOL_F32, assert_normwise, oracle_csrmm_f32, oracle_csrmm_f64,
                     oracle_csrmm_pieces_f32)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ops():
    from spmm_hip import ops
    return ops


def _rand_csr(rng, m, k, deg_hi, hub_rows=(), hub_deg=0, empty_frac=0.0):
    deg = rng.integers(0, deg_hi + 1, m)
    if empty_frac:
        deg[rng.random(m) < empty_frac] = 0
    for r in hub_rows:
        deg[r] = min(hub_deg, k)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(k, d, replace=False)) for d in deg] or
                        [np.zeros(0)]).astype(np.int32)
    val = rng.uniform(-1, 1, ci.size).astype(np.float32)
    return rp, ci, val


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _main_kernel(n: int) -> bool:
    """The launch runs csr_mergepath_kernel (not the K <= 64 lane-group kernel):
    row-major B / C with ld = n, default options."""
    return n > 64 or n % 4 != 0


def _check_rowmajor(oracle, rp, ci, val, B, C, what, exact_expected=False, pieces_exact=None):
    m, n = C.shape
    ref32 = oracle_csrmm_f32(oracle, m, n, rp, ci, val, B, B.shape[1], 0).reshape(m, n)
    ref64, absd = oracle_csrmm_f64(oracle, m, n, rp, ci, val, B, B.shape[1], 0)
    got = C.cpu().numpy()
    assert_normwise(got, ref64, absd, TOL_F32, what + " vs f64")
    assert_normwise(got, ref32.astype(np.float64), absd, TOL_F32, what + " vs seq-f32")
    if exact_expected:
        assert np.array_equal(got, ref32), what + ": expected bit-exact sequential FMA"
    if pieces_exact if pieces_exact is not None else _main_kernel(n):
        pcs = oracle_csrmm_pieces_f32(oracle, m, n, rp, ci, val, B, B.shape[1], 0).reshape(m, n)
        bad = np.flatnonzero(~np.all(got.view(np.uint32) == pcs.view(np.uint32), axis=1))  # bits
        assert bad.size == 0, (f"{what}: {bad.size} rows differ from the piece oracle, "
                               f"first {bad[:5].tolist()}")
    return float(np.mean(got == ref32))


def test_kat_csrmm_cu_via_scsrmm(oracle, golden, device):
    """csrmm.cu:183-185 — cusparseScsrmm, col-major B and C."""
    from spmm_hip._lib import lib
    k = golden["kats"]["csrmm_cu"]
    ops = _ops()
    rp, ci, v = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                     np.array(k["val"], np.float32))
    B = torch.tensor(k["B_colmajor"], dtype=torch.float32, device=device)
    C = torch.zeros(8, dtype=torch.float32, device=device)
    h = ops.default_handle()
    d = ctypes.c_void_p()
    assert lib().spmm_create_mat_descr(ctypes.byref(d)) == 0
    one, zero = ctypes.c_float(1.0), ctypes.c_float(0.0)
    st = lib().spmm_scsrmm(h.raw, 0, 4, 2, 4, 9, ctypes.byref(one), d, ctypes.c_void_p(v.data_ptr()),
                           ctypes.c_void_p(rp.data_ptr()), ctypes.c_void_p(ci.data_ptr()),
                           ctypes.c_void_p(B.data_ptr()), 4, ctypes.byref(zero),
                           ctypes.c_void_p(C.data_ptr()), 4)
    lib().spmm_destroy_mat_descr(d)
    assert st == 0
    assert C.cpu().tolist() == k["C_colmajor"]


def test_kat_csrmm_cu_coo_path(oracle, golden, device):
    """csrmm.cu end to end: its COO rows through cusparseXcoo2csr
    (csrmm.cu:148-149 -> spmm_xcoo2csr), then cusparseScsrmm; both index
    bases; plus a larger row-sorted COO with empty rows against the oracle's
    coo2csr."""
    from helpers import ptr
    k = golden["kats"]["csrmm_cu"]
    ops = _ops()
    for base in (0, 1):
        rows = torch.tensor(np.array(k["coo_row"], np.int32) + base, device=device)
        rp = ops.coo2csr(rows, k["m"], base=base)
        torch.cuda.synchronize()
        assert (rp.cpu().numpy() - base).tolist() == k["rowptr"]
    rp = ops.coo2csr(torch.tensor(np.array(k["coo_row"], np.int32), device=device), k["m"])
    ci, v = _dev(np.array(k["colind"], np.int32), np.array(k["val"], np.float32))
    B = torch.tensor(k["B_colmajor"], dtype=torch.float32, device=device)
    C = torch.zeros(8, dtype=torch.float32, device=device)
    ops.csrmm(rp, ci, v, B, m=4, n=2, k=4, ldb=4, order_b=1, C=C, ldc=4, order_c=1)
    assert C.cpu().tolist() == k["C_colmajor"]
    rng = np.random.default_rng(4)
    m = 100000
    rows = np.sort(rng.integers(0, m, 700000)).astype(np.int32)
    rows = rows[(rows % 7) != 3]  # every seventh row empty
    want = np.zeros(m + 1, np.int32)
    oracle.oracle_coo2csr(ptr(rows), rows.size, m, 0, ptr(want))
    got = ops.coo2csr(torch.from_numpy(rows).to(device), m)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want)


def test_kat_try_cublas_dense_csr(golden, device):
    k = golden["kats"]["try_cublas_cu"]
    ops = _ops()
    rp, ci, v = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                     np.array(k["val"], np.float32))
    B = torch.tensor(k["B_colmajor"], dtype=torch.float32, device=device)
    C = torch.zeros(8, dtype=torch.float32, device=device)
    ops.csrmm(rp, ci, v, B, m=2, n=4, k=3, ldb=3, order_b=1, C=C, ldc=2, order_c=1)
    assert C.cpu().tolist() == k["C_colmajor"]


@pytest.mark.parametrize("shape", [(64, 80, 0.1), (300, 257, 0.03), (1000, 1200, 0.01)])
@pytest.mark.parametrize("K", [32, 64, 100, 128, 256, 512])
def test_gespmm_reference_random_csr(oracle, golden, device, shape, K):
    """randomCSRMatrix fixtures (the reference generator's own output)."""
    m, n, p = shape
    key = f"csr_{m}_{n}_{p}"
    rp, ci, v = (golden["ref"][key + s] for s in ("_rowptr", "_colind", "_val"))
    rng = np.random.default_rng(K)
    B = rng.uniform(-1, 1, (n, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    C = _ops().gespmm_csrmm(drp, dci, dv, dB)
    torch.cuda.synchronize()
    _check_rowmajor(oracle, rp, ci, v, B, C, f"gespmm {key} K={K}")


@pytest.mark.parametrize("K", [1, 2, 4, 7, 8, 16, 28, 32, 64, 128, 130, 256, 512])
def test_power_law_hubs_and_empty_rows(oracle, device, K):
    """Merge-path carries: hub rows spanning many waves, runs of empty rows."""
    rng = np.random.default_rng(100 + K)
    m = 3000
    rp, ci, v = _rand_csr(rng, m, 5000, 6, hub_rows=(0, 1, 1777, m - 1), hub_deg=4000,
                          empty_frac=0.3)
    B = rng.uniform(-1, 1, (5000, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    h = _ops().Handle()
    h.set_csr_waves_per_cu(1)  # few waves -> long merge-path segments
    C = torch.empty((m, K), dtype=torch.float32, device=device)
    _ops().csrmm(drp, dci, dv, dB, n=K, k=5000, ldb=K, C=C, ldc=K, handle=h)
    torch.cuda.synchronize()
    _check_rowmajor(oracle, rp, ci, v, B, C, f"hubs K={K}")
    # differently cut grids give the same bits (pieces: the association is the row's)
    for wpc in (32, 3):
        h.set_csr_waves_per_cu(wpc)
        C2 = torch.empty_like(C)
        _ops().csrmm(drp, dci, dv, dB, n=K, k=5000, ldb=K, C=C2, ldc=K, handle=h)
        torch.cuda.synchronize()
        assert torch.equal(C, C2), f"K={K}: {wpc} waves/CU differs from 1"


def test_unsplit_rows_bit_exact(oracle, device):
    """Small matrix, every row inside one wave: bit-identical to the
    sequential fp32 FMA chain of the reference kernel."""
    rng = np.random.default_rng(5)
    rp, ci, v = _rand_csr(rng, 40, 300, 9)
    B = rng.uniform(-1, 1, (300, 128)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    h = _ops().Handle()
    h.set_csr_waves_per_cu(1)
    C = torch.empty((40, 128), dtype=torch.float32, device=device)
    # one wave for the whole matrix: no carries at all
    _ops().csrmm(drp, dci, dv, dB, n=128, k=300, ldb=128, C=C, ldc=128, handle=h)
    torch.cuda.synchronize()
    frac = _check_rowmajor(oracle, rp, ci, v, B, C, "unsplit", exact_expected=True)
    assert frac == 1.0


@pytest.mark.parametrize("K", [32, 8])
def test_small_k_sequential_rows_option(oracle, device, K):
    """K <= 32 runs the several-rows-per-instruction kernel by default
    (interleaved chains per row, within the fp32 bar); SPMM_CSR_SEQUENTIAL_ROWS
    selects the main kernel, whose unsplit rows are bit-identical to the
    reference's sequential order."""
    from spmm_hip._lib import CSR_NT_STREAMS, CSR_SEQUENTIAL_ROWS
    rng = np.random.default_rng(7)
    rp, ci, v = _rand_csr(rng, 40, 300, 9)
    B = rng.uniform(-1, 1, (300, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    h = _ops().Handle()
    h.set_csr_waves_per_cu(1)
    C = torch.empty((40, K), dtype=torch.float32, device=device)
    h.set_csr_options(CSR_NT_STREAMS | CSR_SEQUENTIAL_ROWS)
    _ops().csrmm(drp, dci, dv, dB, n=K, k=300, ldb=K, C=C, ldc=K, handle=h)
    torch.cuda.synchronize()
    assert _check_rowmajor(oracle, rp, ci, v, B, C, "sequential", exact_expected=True) == 1.0
    h.set_csr_options(CSR_NT_STREAMS)
    C2 = torch.empty_like(C)
    _ops().csrmm(drp, dci, dv, dB, n=K, k=300, ldb=K, C=C2, ldc=K, handle=h)
    torch.cuda.synchronize()
    _check_rowmajor(oracle, rp, ci, v, B, C2, "grouped rows")


@pytest.mark.parametrize("alpha,beta", [(1.0, -0.5), (0.25, 1.0)])
@pytest.mark.parametrize("orders", [(0, 0), (1, 1)])
@pytest.mark.parametrize("K", [4, 12, 32])
def test_small_k_alpha_beta_layouts(oracle, device, alpha, beta, orders, K):
    """The K <= 32 kernel under csrmm semantics: alpha, beta, both storage
    orders, hub rows split across waves (carries), empty rows."""
    ob, oc = orders
    rng = np.random.default_rng(12 + K)
    m, k = 1500, 900
    rp, ci, v = _rand_csr(rng, m, k, 10, hub_rows=(3, 700), hub_deg=800, empty_frac=0.2)
    Bd = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    ldb = K if ob == 0 else k
    C0 = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    Cin = C0 if oc == 0 else np.ascontiguousarray(C0.T)
    ldc = K if oc == 0 else m
    drp, dci, dv, dB, dC = _dev(rp, ci, v, B.reshape(-1), Cin.reshape(-1))
    h = _ops().Handle()
    h.set_csr_waves_per_cu(2)
    _ops().csrmm(drp, dci, dv, dB, n=K, k=k, ldb=ldb, order_b=ob, C=dC, ldc=ldc, order_c=oc,
                 alpha=alpha, beta=beta, handle=h)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape(Cin.shape)
    got = got if oc == 0 else got.T
    ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, Bd, K, 0)
    assert_normwise(got, alpha * ref + beta * C0, abs(alpha) * absd + abs(beta) * np.abs(C0),
                    TOL_F32, f"small K={K} a={alpha} b={beta} orders={orders}")


@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (2.5, 0.0), (1.0, 1.0), (-0.5, 0.75)])
@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1), (1, 0)])
def test_alpha_beta_and_layouts(oracle, device, alpha, beta, orders):
    """cusparseScsrmm / csrmm2 semantics: C = alpha*A*B + beta*C for every
    combination of B / C storage order (run_csrmm.cu:133-142)."""
    ob, oc = orders
    rng = np.random.default_rng(11)
    m, k, n = 333, 401, 96
    rp, ci, v = _rand_csr(rng, m, k, 12, empty_frac=0.1)
    Bd = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    ldb = n if ob == 0 else k
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    Cin = C0 if oc == 0 else np.ascontiguousarray(C0.T)
    ldc = n if oc == 0 else m
    drp, dci, dv, dB, dC = _dev(rp, ci, v, B.reshape(-1), Cin.reshape(-1))
    _ops().csrmm(drp, dci, dv, dB, m=m, n=n, k=k, ldb=ldb, order_b=ob, C=dC, ldc=ldc,
                 order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape(Cin.shape)
    got = got if oc == 0 else got.T
    ref64, absd = oracle_csrmm_f64(oracle, m, n, rp, ci, v, Bd, n, 0)
    ref = alpha * ref64 + beta * C0.astype(np.float64)
    assert_normwise(got, ref, abs(alpha) * absd + abs(beta) * np.abs(C0), TOL_F32,
                    f"alpha={alpha} beta={beta} orders={orders}")


def test_index_base_one(oracle, device):
    rng = np.random.default_rng(3)
    m, k, n = 200, 150, 64
    rp, ci, v = _rand_csr(rng, m, k, 7)
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp + 1, ci + 1, v, B)
    C = torch.empty((m, n), dtype=torch.float32, device=device)
    _ops().csrmm(drp, dci, dv, dB, n=n, k=k, ldb=n, C=C, ldc=n, base=1)
    torch.cuda.synchronize()
    _check_rowmajor(oracle, rp, ci, v, B, C, "base=1")


def test_degenerate_shapes(oracle, device):
    ops = _ops()
    # nnz == 0: every row is an empty row -> zeros
    rp = torch.zeros(51, dtype=torch.int32, device=device)
    ci = torch.zeros(0, dtype=torch.int32, device=device)
    v = torch.zeros(0, dtype=torch.float32, device=device)
    B = torch.randn(10, 64, device=device)
    C = torch.full((50, 64), 7.0, device=device)
    ops.csrmm(rp, ci, v, B, n=64, k=10, ldb=64, C=C, ldc=64)
    torch.cuda.synchronize()
    assert torch.count_nonzero(C).item() == 0
    # m == 0 is a quick return
    C0 = torch.zeros(0, 64, device=device)
    ops.csrmm(torch.zeros(1, dtype=torch.int32, device=device), ci, v, B, n=64, k=10, ldb=64,
              C=C0, ldc=64)


def test_status_codes(device):
    from spmm_hip._lib import INVALID_VALUE, MATRIX_TYPE_NOT_SUPPORTED, NOT_INITIALIZED, lib
    L = lib()
    one = ctypes.c_float(1.0)
    assert L.spmm_csrmm_ex_f32(None, 1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0,
                               None, 1, 0) == NOT_INITIALIZED
    h = _ops().default_handle()
    assert L.spmm_csrmm_ex_f32(h.raw, -1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0,
                               None, 1, 0) == INVALID_VALUE
    d = ctypes.c_void_p()
    L.spmm_create_mat_descr(ctypes.byref(d))
    assert L.spmm_scsrmm(h.raw, 1, 4, 2, 4, 9, ctypes.byref(one), d, None, None, None, None, 4,
                         ctypes.byref(one), None, 4) == MATRIX_TYPE_NOT_SUPPORTED
    L.spmm_destroy_mat_descr(d)


def test_products_scale_properties(oracle, device):
    """BASELINE full size (ogbn-products stand-in, K=128): a sample of rows
    against the oracle, determinism, and linearity A(B1+B2) = AB1 + AB2."""
    from spmm_hip import prep
    n, nnz, K = 2449029, 61859140, 128
    rp, ci = prep.powerlaw_csr(n, nnz, 17481, 2.3, 1234)
    rng = np.random.default_rng(0)
    v = rng.uniform(-1, 1, nnz).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    B1 = torch.rand((n, K), device=device) * 2 - 1
    B2 = torch.rand((n, K), device=device) * 2 - 1
    ops = _ops()
    C1 = ops.gespmm_csrmm(drp, dci, dv, B1)
    C1b = ops.gespmm_csrmm(drp, dci, dv, B1)
    C2 = ops.gespmm_csrmm(drp, dci, dv, B2)
    C12 = ops.gespmm_csrmm(drp, dci, dv, B1 + B2)
    torch.cuda.synchronize()
    assert torch.equal(C1, C1b), "not deterministic"
    # sampled rows (hub rows included) vs the f64 oracle
    deg = np.diff(rp)
    rows = np.unique(np.concatenate([rng.choice(n, 2000, replace=False),
                                     np.argsort(deg)[-20:]]))
    sub_rp = np.concatenate([[0], np.cumsum(deg[rows])]).astype(np.int32)
    sub_ci = np.concatenate([ci[rp[r]:rp[r + 1]] for r in rows]).astype(np.int32)
    sub_v = np.concatenate([v[rp[r]:rp[r + 1]] for r in rows]).astype(np.float32)
    Bh = B1.cpu().numpy()
    ref64, absd = oracle_csrmm_f64(oracle, rows.size, K, sub_rp, sub_ci, sub_v, Bh, K, 0)
    assert_normwise(C1.cpu().numpy()[rows], ref64, absd, TOL_F32, "products rows")
    # linearity within the same tolerance (sum of the two magnitudes)
    lin = (C1 + C2 - C12).abs()
    absd_full = ops.gespmm_csrmm(drp, dci, dv.abs(), B1.abs() + B2.abs())
    assert bool((lin <= 3 * TOL_F32 * absd_full + 1e-30).all())


@pytest.mark.parametrize("K", [128, 32, 36])
def test_row_shards_match_whole_matrix(oracle, device, K):
    """SURVEY §8e on one device: the rows of each nnz-balanced shard computed
    alone equal the whole-matrix result bit for bit (main kernel at K = 128 /
    36, lane-group kernel at K = 32 on residue-preserving shard arrays)."""
    from spmm_hip import dist as sdist
    rng = np.random.default_rng(21)
    m, k = 6000, 6000
    rp, ci, v = _rand_csr(rng, m, k, 20, hub_rows=(10, 2500, 5999), hub_deg=3000)
    B = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    Cw = torch.empty((m, K), dtype=torch.float32, device=device)
    _ops().csrmm(drp, dci, dv, dB, n=K, k=k, ldb=K, C=Cw, ldc=K)
    parts = []
    for world in (2, 3, 8):
        for r in range(world):
            sh = sdist.make_shard(rp, ci, v, r, world)
            srp, sci, sv = _dev(sh.rowptr, np.ascontiguousarray(sh.colind),
                                np.ascontiguousarray(sh.val))
            Cs = torch.empty((sh.rows, K), dtype=torch.float32, device=device)
            if sh.rows:
                _ops().csrmm(srp, sci, sv, dB, m=sh.rows, n=K, k=k, ldb=K, C=Cs, ldc=K)
            parts.append((sh.row0, sh.row1, Cs))
    torch.cuda.synchronize()
    whole = Cw.cpu().numpy()
    ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, B, K, 0)
    for r0, r1, Cs in parts:
        got = Cs.cpu().numpy()
        assert_normwise(got, ref[r0:r1], absd[r0:r1], TOL_F32, f"shard {r0}:{r1}")
        same = np.all(got == whole[r0:r1], axis=1)
        assert same.all(), (r0, r1, np.flatnonzero(~same)[:5])


def test_permutation_invariance(oracle, device):
    """(P A P^T)(P B) = P (A B) through the reorder front-end."""
    from spmm_hip import prep
    rng = np.random.default_rng(22)
    rp, ci = prep.community_csr(4000, 25.0, 32, 128, 0.9, 5)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    n, K = rp.size - 1, 64
    B = rng.uniform(-1, 1, (n, K)).astype(np.float32)
    o2n = prep.reorder(rp, ci, "rcm")
    prp, pci, pv = prep.permute_csr(rp, ci, o2n, v)
    PB = np.empty_like(B)
    PB[o2n] = B
    d1 = _dev(rp, ci, v, B)
    d2 = _dev(prp, pci, pv, PB)
    C1 = torch.empty((n, K), dtype=torch.float32, device=device)
    C2 = torch.empty((n, K), dtype=torch.float32, device=device)
    _ops().csrmm(*d1, n=K, k=n, ldb=K, C=C1, ldc=K)
    _ops().csrmm(*d2, n=K, k=n, ldb=K, C=C2, ldc=K)
    torch.cuda.synchronize()
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, B, K, 0)
    got = np.empty_like(B)
    got[:] = C2.cpu().numpy()[o2n]  # row o2n[i] of the permuted product is row i
    assert_normwise(got, ref, absd, TOL_F32, "P A P^T (P B)")
    assert_normwise(C1.cpu().numpy(), ref, absd, TOL_F32, "A B")


@pytest.mark.parametrize("m,K,beta", [(200_000, 128, 0.0), (200_003, 64, 0.5), (70_001, 130, -1.0)])
def test_colmajor_forms_match_rowmajor(device, m, K, beta):
    """cusparseScsrmm's layout (run_csrmm.cu:135-137: column-major B and C) at
    sizes where the staging transposes run many tiles, edge tiles and both the
    16-byte and the scalar transpose kernels: B transposed and C transposed
    back are exact copies, the product is the same kernel and the transpose's
    fma(beta, C, x) is the kernel's own epilogue, so the result is bit-identical
    to the row-major call at every beta."""
    from spmm_hip import prep
    ops = _ops()
    rp, ci = prep.powerlaw_csr(m, 12 * m, 3000, 2.3, 3)
    rng = np.random.default_rng(m + K)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    B = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    drp, dci, dv, dB, dC = _dev(rp, ci, v, B, C0)
    ops.csrmm(drp, dci, dv, dB, n=K, k=m, ldb=K, C=dC, ldc=K, beta=beta)
    dBc = dB.t().contiguous()
    dCc = torch.from_numpy(np.ascontiguousarray(C0.T)).cuda()
    ops.csrmm(drp, dci, dv, dBc, n=K, k=m, ldb=m, order_b=ops.ORDER_COL, C=dCc, ldc=m,
              order_c=ops.ORDER_COL, beta=beta)
    torch.cuda.synchronize()
    assert torch.equal(dCc.t(), dC)


@pytest.mark.parametrize("K,opts,alpha,beta", [
    (128, 0, 1.0, 0.0), (512, 0, 1.0, 0.0), (256, 0, 1.0, 0.0), (32, 2, 1.0, 0.0),
    (64, 0, 1.0, 0.0), (128, 0, 2.0, 0.5), (512, 0, -0.5, 2.0), (256, 0, 0.25, -1.0),
    (32, 2, 2.0, -0.5), (64, 0, -2.0, 0.5), (64, 0, 0.7, -1.3), (128, 0, 0.7, -1.3),
    (130, 0, 0.7, -1.3), (36, 0, 1.0, 0.0)])
def test_split_rows_bit_exact_pieces(oracle, device, K, opts, alpha, beta):
    """Every row, split over waves or not, is bit-identical to the piece oracle
    (oracle_csrmm_pieces_f32): pieces of a split row stored by their waves and
    added in piece order by the last arrival (split-row tickets,
    csr_kernels.hip), at any alpha / beta (a finite C0 read by the finishing
    wave). Power-law rows with hubs spanning dozens of waves, empty rows, K at
    every vector width of the main kernel (K = 32 with SPMM_CSR_SEQUENTIAL_ROWS);
    K = 64 / 36 run the lane-group kernel, whose pieces are interleaved chains:
    within the bar, and the same bits at every grid."""
    from spmm_hip import prep
    from spmm_hip._lib import CSR_NT_STREAMS
    ops = _ops()
    m, nnz = 40000, 600000
    rp, ci = prep.powerlaw_csr(m, nnz, 15000, 2.1, 11)
    v = np.random.default_rng(3).uniform(-1, 1, ci.size).astype(np.float32)
    B = np.random.default_rng(4).uniform(-1, 1, (m, K)).astype(np.float32)
    C0 = np.random.default_rng(5).uniform(-1, 1, (m, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    h = ops.Handle()
    h.set_csr_options(CSR_NT_STREAMS | opts)
    init = (lambda: torch.from_numpy(C0).to(device)) if beta != 0.0 else \
        (lambda: torch.full((m, K), float("nan"), device=device))
    C = init()
    ops.csrmm(drp, dci, dv, dB, n=K, k=m, ldb=K, C=C, ldc=K, alpha=alpha, beta=beta, handle=h)
    torch.cuda.synchronize()
    got = C.cpu().numpy()
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    nwaves = min(-(-(m + ci.size) // 256), cus * 16)  # kMinItemsPerWave, csr_kernels.hip
    per = -(-(m + ci.size) // nwaves)
    split = np.array([(r + rp[r]) // per != (r + rp[r + 1]) // per for r in range(m)])
    assert split.sum() > 50, "the case must split many rows"
    if not _main_kernel(K) and not opts:  # the lane-group kernel
        ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, B, K, 0)
        ref = alpha * ref + beta * C0.astype(np.float64)
        absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
        assert_normwise(got, ref, absd, TOL_F32, f"K={K} alpha={alpha} beta={beta}, split rows")
        want = got
    else:
        want = oracle_csrmm_pieces_f32(oracle, m, K, rp, ci, v, B, K, 0, alpha=alpha, beta=beta,
                                       C=C0).reshape(m, K)
        bad = got.view(np.uint32) != want.view(np.uint32)  # bits, signed zeros included
        assert not bad.any(), (f"K={K}: {int(bad.any(axis=1).sum())} rows differ from the piece "
                               f"oracle ({int(bad[split].any(axis=1).sum())} of "
                               f"{int(split.sum())} split rows)")
    # repeated launches (tickets back at zero after every launch) and other grids
    for wpc in (16, 16, 1, 5, 32):
        h.set_csr_waves_per_cu(wpc)
        C = init()
        ops.csrmm(drp, dci, dv, dB, n=K, k=m, ldb=K, C=C, ldc=K, alpha=alpha, beta=beta,
                  handle=h)
        torch.cuda.synchronize()
        assert np.array_equal(C.cpu().numpy(), want), f"{wpc} waves/CU differs"
    h.close()


def test_dropin_equals_ex_entry(device):
    """gespmm_csrmm (grid sized without nnz) and spmm_csrmm_ex_f32 (grid from
    nnz) give the same bits: the association is the row's, not the grid's."""
    from spmm_hip import prep
    ops = _ops()
    for m, nnz, K in ((20000, 400000, 128), (20000, 400000, 32), (6000, 900000, 256)):
        rp, ci = prep.powerlaw_csr(m, nnz, m // 2, 2.1, 5)
        v = np.random.default_rng(6).uniform(-1, 1, ci.size).astype(np.float32)
        B = np.random.default_rng(7).uniform(-1, 1, (m, K)).astype(np.float32)
        drp, dci, dv, dB = _dev(rp, ci, v, B)
        Cd = ops.gespmm_csrmm(drp, dci, dv, dB)
        Cx = torch.empty_like(Cd)
        ops.csrmm(drp, dci, dv, dB, n=K, k=m, ldb=K, C=Cx, ldc=K)
        torch.cuda.synchronize()
        assert torch.equal(Cd, Cx), (m, nnz, K)


@pytest.mark.parametrize("seed", range(12))
def test_random_shapes_grid_independent(oracle, device, seed):
    """Random matrices (rows of 0 .. 3,000 nonzeros, hubs up to 9,000, empty rows),
    random K among every kernel's widths, random alpha / beta and two random grids
    (waves per CU 1 .. 32): the main kernel equals the piece oracle bit for bit at
    both grids, the K <= 64 lane-group kernel gives the same bits at both grids and
    is within the fp32 bar of the f64 product."""
    ops = _ops()
    rng = np.random.default_rng(7000 + seed)
    m = int(rng.integers(1, 30000))
    k = int(rng.integers(1, 20000))
    K = int(rng.choice([1, 4, 8, 12, 16, 32, 36, 64, 96, 128, 130, 192, 256, 512]))
    nhub = int(rng.integers(0, 6))
    hubs = rng.choice(m, min(nhub, m), replace=False) if nhub else ()
    rp, ci, v = _rand_csr(rng, m, k, min(int(rng.choice([0, 3, 20, 200, 3000])), k), hubs,
                          int(rng.integers(1000, 9001)), float(rng.choice([0.0, 0.3])))
    alpha = float(rng.choice([1.0, -0.5, 2.0]))
    beta = float(rng.choice([0.0, 0.0, 0.75]))
    B = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    got = []
    for wpc in rng.choice(np.arange(1, 33), 2, replace=False):
        h = ops.Handle()
        h.set_csr_waves_per_cu(int(wpc))
        C = torch.from_numpy(C0).to(device)
        ops.csrmm(drp, dci, dv, dB, n=K, k=k, ldb=K, C=C, ldc=K, alpha=alpha, beta=beta, handle=h)
        torch.cuda.synchronize()
        got.append(C.cpu().numpy())
        h.close()
    what = f"m={m} k={k} K={K} nnz={ci.size} alpha={alpha} beta={beta}"
    assert np.array_equal(got[0].view(np.uint32), got[1].view(np.uint32)), what + ": grids differ"
    # row shards (dist.make_shard: positions mod 64 kept) written in place: the same bits,
    # the lane-group kernel's too
    from spmm_hip import dist as sdist
    for world in (2, 3):
        Cs = torch.from_numpy(C0).to(device)
        for r in range(world):
            sh = sdist.make_shard(rp, ci, v, r, world)
            if sh.rows == 0:
                continue
            srp, sci, sv = _dev(sh.rowptr, sh.colind, sh.val)
            ops.csrmm(srp, sci, sv, dB, m=sh.rows, n=K, k=k, ldb=K, C=Cs[sh.row0:sh.row1], ldc=K,
                      alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        assert np.array_equal(Cs.cpu().numpy().view(np.uint32), got[0].view(np.uint32)), \
            f"{what}: {world} shards"
    # the column-major forms (cusparseScsrmm2's layout: staged through LDS-tiled transposes,
    # the epilogue the kernel's own) give the same bits
    dBc = torch.from_numpy(np.ascontiguousarray(B.T)).to(device)
    Cc = torch.from_numpy(np.ascontiguousarray(C0.T)).to(device)
    ops.csrmm(drp, dci, dv, dBc, m=m, n=K, k=k, ldb=k, order_b=ops.ORDER_COL, C=Cc, ldc=m,
              order_c=ops.ORDER_COL, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    colm = np.ascontiguousarray(Cc.cpu().numpy().T)
    if _main_kernel(K):
        assert np.array_equal(colm.view(np.uint32), got[0].view(np.uint32)), what + ": column-major"
        # the hot-column entry (a small budget, so some columns go each way): the same bits
        tag = ops.csr_hot_analysis(dci, n=K, k=k, hot_bytes=int(rng.choice([1 << 12, 1 << 20])))
        Ch = torch.from_numpy(C0).to(device)
        ops.csrmm_hot(drp, tag, dv, dB, m=m, n=K, k=k, ldb=K, C=Ch, ldc=K, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        assert np.array_equal(Ch.cpu().numpy().view(np.uint32), got[0].view(np.uint32)), \
            what + ": hot-column entry"
    if _main_kernel(K):
        want = oracle_csrmm_pieces_f32(oracle, m, K, rp, ci, v, B, K, 0, alpha=alpha, beta=beta,
                                       C=C0).reshape(m, K)
        bad = got[0].view(np.uint32) != want.view(np.uint32)
        assert not bad.any(), f"{what}: {int(bad.sum())} elements differ from the piece oracle"
    else:
        ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, B, K, 0)
        ref = alpha * ref + beta * C0.astype(np.float64)
        absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
        assert_normwise(got[0], ref, absd, TOL_F32, what)
