"""fp64 forms of both paths (T = double in gespmm_csrmm<T>, gespmm_csrmm.h:422,
and rocsparse_bsrmm_template<T>, rocsparse_bsrmm.h:102) through the C ABI vs
the fp64 oracle.

Bar: bit-exact. The fp64 kernels run one sequential FMA chain per output
element in the oracle's order (CSR order; blocks in order, q = 0..bs-1), with
the same alpha/beta epilogue, so every element must match exactly."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from helpers import oracle_bsrmm_d, oracle_csrmm_d

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ops():
    from spmm_hip import ops
    return ops


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _csr(rng, m, k, deg_hi, empty_frac=0.1):
    deg = rng.integers(0, deg_hi + 1, m)
    deg[rng.random(m) < empty_frac] = 0
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(k, d, replace=False)) for d in deg]).astype(np.int32)
    return rp, ci, rng.standard_normal(ci.size)


def _bsr(rng, mb, kb, bs, p):
    mask = rng.random((mb, kb)) < p
    brp = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
    bci = np.nonzero(mask)[1].astype(np.int32)
    return brp, bci, rng.standard_normal(bci.size * bs * bs)


@pytest.mark.parametrize("n", [1, 7, 64, 130])
@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("alpha,beta,base", [(1.0, 0.0, 0), (0.75, -1.5, 1)])
def test_csrmm_f64(oracle, device, n, orders, alpha, beta, base):
    rng = np.random.default_rng(n * 7 + orders[0] * 2 + orders[1])
    m, k = 517, 389
    rp, ci, v = _csr(rng, m, k, 40)
    ob, oc = orders
    B = rng.standard_normal((k, n) if ob == 0 else (n, k))
    C0 = rng.standard_normal((m, n) if oc == 0 else (n, m))
    ldb, ldc = (n if ob == 0 else k), (n if oc == 0 else m)
    ref = oracle_csrmm_d(oracle, m, n, rp + base, ci + base, v, B, ldb, ob, alpha, beta,
                         C0.ravel(), ldc, oc, base)
    drp, dci, dv, dB, dC = _dev(rp + base, ci + base, v, B, C0)
    _ops().csrmm(drp, dci, dv, dB, m=m, n=n, k=k, ldb=ldb, order_b=ob, C=dC, ldc=ldc,
                 order_c=oc, alpha=alpha, beta=beta, base=base)
    assert np.array_equal(dC.cpu().numpy().ravel(), ref)


def test_gespmm_csrmm_double(oracle, device):
    """gespmm_csrmm<double>: row-major B and C, C overwritten."""
    rng = np.random.default_rng(11)
    m, k, n = 2000, 1500, 96
    rp, ci, v = _csr(rng, m, k, 60)
    B = rng.standard_normal((k, n))
    ref = oracle_csrmm_d(oracle, m, n, rp, ci, v, B, n, 0)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    C = _ops().gespmm_csrmm(drp, dci, dv, dB)
    assert C.dtype == torch.float64
    assert np.array_equal(C.cpu().numpy().ravel(), ref)


@pytest.mark.parametrize("bs", [1, 2, 3, 8, 16, 32, 64])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1)])
def test_bsrmm_f64(oracle, device, bs, direction, orders):
    rng = np.random.default_rng(bs * 10 + direction)
    mb, kb, n = 23, 19, 70
    brp, bci, bv = _bsr(rng, mb, kb, bs, 0.25)
    ob, oc = orders
    m, k = mb * bs, kb * bs
    B = rng.standard_normal((k, n) if ob == 0 else (n, k))
    C0 = rng.standard_normal((m, n) if oc == 0 else (n, m))
    ldb, ldc = (n if ob == 0 else k), (n if oc == 0 else m)
    ref = oracle_bsrmm_d(oracle, direction, mb, n, bs, brp, bci, bv, B, ldb, ob, 0.5, 2.0,
                         C0.ravel(), ldc, oc)
    dbrp, dbci, dbv, dB, dC = _dev(brp, bci, bv, B, C0)
    _ops().bsrmm(dbrp, dbci, dbv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, order_b=ob, C=dC,
                 ldc=ldc, order_c=oc, alpha=0.5, beta=2.0, direction=direction)
    assert np.array_equal(dC.cpu().numpy().ravel(), ref)


def test_dcsrmm2_dbsrmm_cusparse_shapes(oracle, golden, device):
    """cusparseDcsrmm2 / cusparseDbsrmm call shapes (col-major C, transB) on the
    reference's KAT operands (csrmm.cu, bsrmm.cu) in double."""
    from spmm_hip._lib import lib
    ops = _ops()
    h = ops.default_handle()
    d = ctypes.c_void_p()
    assert lib().spmm_create_mat_descr(ctypes.byref(d)) == 0
    one, zero = ctypes.c_double(1.0), ctypes.c_double(0.0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    try:
        k = golden["kats"]["csrmm_cu"]
        rp, ci, v = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                         np.array(k["val"], np.float64))
        B = torch.tensor(k["B_colmajor"], dtype=torch.float64, device=device)
        C = torch.zeros(len(k["C_colmajor"]), dtype=torch.float64, device=device)
        st = lib().spmm_dcsrmm2(h.raw, 0, 0, k["m"], k["n"], k["k"],
                                ci.numel(), ctypes.byref(one), d, P(v), P(rp), P(ci), P(B),
                                k["ldb"], ctypes.byref(zero), P(C), k["ldc"])
        assert st == 0
        assert C.cpu().tolist() == k["C_colmajor"]
        k = golden["kats"]["bsrmm_cu"]
        brp, bci, bv = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                            np.array(k["val"], np.float64))
        B = torch.tensor(k["B_colmajor"], dtype=torch.float64, device=device)
        C = torch.zeros(len(k["C_colmajor"]), dtype=torch.float64, device=device)
        st = lib().spmm_dbsrmm(h.raw, k["dir"], 0, 0, k["mb"], k["n"], k["kb"], bci.numel(),
                               ctypes.byref(one), d, P(bv), P(brp), P(bci), k["bs"], P(B),
                               k["ldb"], ctypes.byref(zero), P(C), k["ldc"])
        assert st == 0
        assert C.cpu().tolist() == k["C_colmajor"]
    finally:
        lib().spmm_destroy_mat_descr(d)


def test_f64_status_codes(device):
    from spmm_hip._lib import lib
    ops = _ops()
    h = ops.default_handle()
    z = ctypes.c_void_p(0)
    # bad order / negative sizes / ldb too small
    assert lib().spmm_csrmm_ex_f64(h.raw, 4, 4, 4, 0, 1.0, z, z, z, 0, z, 4, 7, 0.0, z, 4,
                                   0) == 3
    assert lib().spmm_csrmm_ex_f64(h.raw, -1, 4, 4, 0, 1.0, z, z, z, 0, z, 4, 0, 0.0, z, 4,
                                   0) == 3
    rp, B, C = _dev(np.zeros(5, np.int32), np.zeros(16), np.zeros(16))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib().spmm_csrmm_ex_f64(h.raw, 4, 4, 4, 0, 1.0, P(rp), z, z, 0, P(B), 3, 0, 0.0,
                                   P(C), 4, 0) == 3
    # empty matrix: C = alpha*0 + beta*C
    assert lib().spmm_csrmm_ex_f64(h.raw, 4, 4, 4, 0, 1.0, P(rp), z, z, 0, P(B), 4, 0, 0.0,
                                   P(C), 4, 0) == 0
    torch.cuda.synchronize()
    assert not C.any()
    assert lib().spmm_bsrmm_ex_f64(h.raw, 5, 1, 1, 4, 0, 4, 1.0, z, z, z, z, 4, 0, 0.0, z, 4,
                                   0) == 3
    with pytest.raises(TypeError):
        ops.csrmm(rp, rp[:0], torch.zeros(0, device=device), B, n=4, k=4, ldb=4, C=C, ldc=4)


@pytest.mark.parametrize("seed", range(8))
def test_random_shapes_f64_bits(oracle, device, seed):
    """fp64 CSR and BSR forms on random shapes (empty rows, K 1 to 300, bs 1 to 32,
    both storage orders, random alpha / beta): bit for bit, signed zeros included,
    the sequential fp64 oracles; the device csr2bsr of the same matrix equals the
    host conversion bit for bit."""
    from spmm_hip import prep
    ops = _ops()
    rng = np.random.default_rng(9500 + seed)
    m, k = int(rng.integers(1, 3000)), int(rng.integers(1, 3000))
    K = int(rng.choice([1, 3, 16, 64, 100, 128, 300]))
    rp, ci, v = _csr(rng, m, k, min(int(rng.choice([0, 4, 40, 400])), k))
    alpha, beta = float(rng.choice([1.0, -1.5])), float(rng.choice([0.0, 0.25]))
    B = rng.standard_normal((k, K))
    C0 = rng.standard_normal((m, K))
    order = int(rng.integers(0, 2))
    drp, dci, dv = _dev(rp, ci, v)
    if order == 0:
        dB, dC = _dev(B, C0.copy())
        ops.csrmm(drp, dci, dv, dB, m=m, n=K, k=k, ldb=K, C=dC, ldc=K, alpha=alpha, beta=beta)
        got = dC.cpu().numpy()
    else:
        dB, dC = _dev(np.ascontiguousarray(B.T), np.ascontiguousarray(C0.T))
        ops.csrmm(drp, dci, dv, dB, m=m, n=K, k=k, ldb=k, order_b=ops.ORDER_COL, C=dC, ldc=m,
                  order_c=ops.ORDER_COL, alpha=alpha, beta=beta)
        got = dC.cpu().numpy().T
    want = oracle_csrmm_d(oracle, m, K, rp, ci, v, B, K, 0, alpha=alpha, beta=beta,
                          C=C0.copy().reshape(-1)).reshape(m, K)
    what = f"f64 csr m={m} k={k} K={K} order={order} alpha={alpha} beta={beta}"
    assert np.array_equal(np.ascontiguousarray(got).view(np.int64), want.view(np.int64)), what
    # the same matrix in blocks: device csr2bsr against the host one, then the fp64 BSR form
    bs = int(rng.choice([1, 2, 4, 8, 16, 32]))
    hb = prep.csr2bsr(m, k, rp, ci, v.astype(np.float32), bs)
    db = ops.csr2bsr(drp, dci, dv.float(), m=m, n=k, bs=bs)
    for h, d, nm in zip(hb, db, ("rowptr", "colind", "values")):
        assert np.array_equal(h.view(np.int32), d.cpu().numpy().view(np.int32)), f"csr2bsr {nm}"
    brp, bci, bv32 = hb
    mb, kb = (m + bs - 1) // bs, (k + bs - 1) // bs
    bv = bv32.astype(np.float64)
    Bp = np.zeros((kb * bs, K))
    Bp[:k] = B
    Cp = np.zeros((mb * bs, K))
    Cp[:m] = C0
    d1, d2, d3, dBp, dCp = _dev(brp, bci, bv, Bp, Cp.copy())
    ops.bsrmm(d1, d2, d3, dBp, mb=mb, kb=kb, n=K, bs=bs, ldb=K, C=dCp, ldc=K, alpha=alpha, beta=beta)
    wantb = oracle_bsrmm_d(oracle, 0, mb, K, bs, brp, bci, bv, Bp, K, 0, alpha=alpha, beta=beta,
                           C=Cp.copy().reshape(-1)).reshape(mb * bs, K)
    if bci.size == 0:  # rocsparse_bsrmm.h:152-154's quick return: C untouched, beta or not
        wantb = Cp
    assert np.array_equal(dCp.cpu().numpy().view(np.int64), wantb.view(np.int64)), \
        f"f64 bsr bs={bs} {what}"
