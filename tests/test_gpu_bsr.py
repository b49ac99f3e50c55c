"""Path B parity on the GPU: BSR x dense (fp32 MFMA, fp16 MFMA, generic)
through the C ABI vs the oracle, with cusparseSbsrmm semantics."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from helpers import (TOL_F16_ACC, TOL_F32, assert_normwise, oracle_bsrmm_f32, oracle_bsrmm_f64,
                     oracle_csrmm_f64)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ops():
    from spmm_hip import ops
    return ops


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _rand_bsr(rng, mb, kb, bs, p, empty_rows=()):
    rows = []
    for br in range(mb):
        cols = np.nonzero(rng.random(kb) < p)[0] if br not in empty_rows else np.zeros(0, int)
        rows.append(cols)
    rp = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32) if rp[-1] else np.zeros(0, np.int32)
    val = rng.uniform(-1, 1, rp[-1] * bs * bs).astype(np.float32)
    return rp, ci, val


def test_kat_bsrmm_cu_via_sbsrmm(golden, device):
    """bsrmm.cu:141-144: cusparseSbsrmm ROW, transB = N (col-major B, C)."""
    from spmm_hip._lib import lib
    k = golden["kats"]["bsrmm_cu"]
    rp, ci, v = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                     np.array(k["val"], np.float32))
    B = torch.tensor(k["B_colmajor"], dtype=torch.float32, device=device)
    C = torch.zeros(8, dtype=torch.float32, device=device)
    h = _ops().default_handle()
    d = ctypes.c_void_p()
    lib().spmm_create_mat_descr(ctypes.byref(d))
    one, zero = ctypes.c_float(1.0), ctypes.c_float(0.0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    st = lib().spmm_sbsrmm(h.raw, 0, 0, 0, k["mb"], k["n"], k["kb"], 4, ctypes.byref(one), d,
                           P(v), P(rp), P(ci), k["bs"], P(B), k["ldb"], ctypes.byref(zero), P(C),
                           k["ldc"])
    lib().spmm_destroy_mat_descr(d)
    assert st == 0
    assert C.cpu().tolist() == k["C_colmajor"]


def test_kat_block_cublas(golden, device):
    """block_cublas.cu:123-136 per-block cublasSgemm == dir COLUMN, row-major
    B, col-major C, beta = 1 onto zeroed C."""
    k = golden["kats"]["block_cublas_cu"]
    rp, ci, v = _dev(np.array(k["rowptr"], np.int32), np.array(k["colind"], np.int32),
                     np.array(k["val"], np.float32))
    B = torch.tensor(k["B_rowmajor"], dtype=torch.float32, device=device)
    C = torch.zeros(12, dtype=torch.float32, device=device)
    _ops().bsrmm(rp, ci, v, B, mb=k["mb"], kb=k["kb"], n=k["n"], bs=k["bs"], ldb=k["ldb"],
                 order_b=0, C=C, ldc=k["ldc"], order_c=1, beta=k["beta"], direction=k["dir"])
    assert C.cpu().tolist() == k["C_colmajor"]


def test_reference_random_bsr_fixture(oracle, golden, device):
    """randomBSRMatrix's own output (load_data.cc:81-113, compiled from the
    reference into oracle/_ref: ref_host.npz bsr_12_10_4) through
    cusparseSbsrmm's shapes, both B layouts, against the oracle."""
    r = golden["ref"]
    rp, ci, v = r["bsr_12_10_4_rowptr"], r["bsr_12_10_4_colind"], r["bsr_12_10_4_val"]
    mb, kb, bs = 12, 10, 4
    for n, ob in ((7, 0), (64, 1)):
        B = np.random.default_rng(n).uniform(-1, 1, (kb * bs, n)).astype(np.float32)
        Bl = B if ob == 0 else np.ascontiguousarray(B.T)
        drp, dci, dv, dB = _dev(rp, ci, v, Bl)
        C = torch.zeros((n, mb * bs), dtype=torch.float32, device=device)  # col-major
        _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n if ob == 0 else kb * bs,
                     order_b=ob, C=C, ldc=mb * bs, order_c=1)
        torch.cuda.synchronize()
        ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
        assert_normwise(C.cpu().numpy().T, ref, absd, TOL_F32, f"randomBSRMatrix n={n}")


@pytest.mark.parametrize("bs,p,n", [(16, 0.05, 128), (32, 0.05, 128), (16, 0.1, 512)])
def test_reference_generator_bsr_on_mfma(oracle, device, bs, p, n):
    """randomBSRMatrix from the library's host generator (bit-exact with the
    reference's, tests/test_prep.py) at the MFMA block sizes, row-major B and
    C (the shipped kernels) and fp16 at bs 16."""
    from spmm_hip import prep
    mb = 4096 // bs
    prep.rng_seed(1234)
    rp, ci, v = prep.random_bsr(mb, mb, bs, p)
    B = prep.random_dense_matrix(mb * bs, n)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    C = torch.empty((mb * bs, n), dtype=torch.float32, device=device)
    _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=mb, n=n, bs=bs, ldb=n, C=C, ldc=n)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F32, f"random_bsr bs={bs} fp32")
    if bs == 16:
        v16, B16 = v.astype(np.float16), B.astype(np.float16)
        C16 = torch.empty((mb * bs, n), dtype=torch.float32, device=device)
        _ops().bsrmm_f16(drp, dci, dv.half(), dB.half(), mb=mb, kb=mb, n=n, bs=bs, ldb=n, C=C16,
                         ldc=n)
        torch.cuda.synchronize()
        ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v16, B16, n, 0, half=True)
        assert_normwise(C16.cpu().numpy(), ref, absd, TOL_F16_ACC, "random_bsr bs=16 fp16")


@pytest.mark.parametrize("bs", [2, 3, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1)])
def test_bsrmm_f32(oracle, device, bs, direction, orders):
    ob, oc = orders
    rng = np.random.default_rng(bs * 10 + direction)
    mb, kb = 23, 29
    n = 130 if bs <= 16 else 96
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.2, empty_rows=(3, 4))
    K = kb * bs
    Bd = rng.uniform(-1, 1, (K, n)).astype(np.float32)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    ldb = n if ob == 0 else K
    m = mb * bs
    ldc = n if oc == 0 else m
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    C = torch.full((m * n,), float("nan"), device=device)
    _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, order_b=ob, C=C, ldc=ldc,
                 order_c=oc, direction=direction)
    torch.cuda.synchronize()
    got = C.cpu().numpy().reshape((m, n) if oc == 0 else (n, m))
    got = got if oc == 0 else got.T
    ref, absd = oracle_bsrmm_f64(oracle, direction, mb, n, bs, rp, ci, v, Bd, n, 0)
    assert_normwise(got, ref, absd, TOL_F32, f"bsr bs={bs} dir={direction} orders={orders}")


@pytest.mark.parametrize("cpad,coff", [(1, 0), (4, 1), (0, 2)])
def test_bsrmm_f32_bs32_unaligned_row_major_c(oracle, device, cpad, coff):
    """Row-major C whose rows are not 16-B aligned (odd ldc, or C starting 1 or
    2 floats into its buffer): the bs 32 column stream stores 16-B row pieces,
    so these calls take the fragment kernel's scalar stores; alpha / beta and
    the padding columns are checked."""
    rng = np.random.default_rng(41 + cpad + 7 * coff)
    mb, kb, bs, n = 19, 27, 32, 136
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.3, empty_rows=(2,))
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    m, ldc = mb * bs, n + cpad
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    Cm = np.full(coff + m * ldc, 7.0, np.float32)
    Cm[coff:].reshape(m, ldc)[:, :n] = C0
    drp, dci, dv, dB, dC = _dev(rp, ci, v, B.reshape(-1), Cm)
    alpha, beta = -0.75, 0.5
    _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC[coff:], ldc=ldc,
                 alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    out = dC.cpu().numpy()
    got = out[coff:].reshape(m, ldc)
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(got[:, :n], ref, absd, TOL_F32, f"bs32 cpad={cpad} coff={coff}")
    assert np.all(got[:, n:] == 7.0) and np.all(out[:coff] == 7.0)


def test_segments_with_staged_col_major_b(oracle, device):
    """Column-major B is staged (transposed) into the handle workspace before
    the bs 32 column stream runs; on a shallow grid with one long block row
    that kernel also splits the row into segments whose partial tiles need
    scratch memory. The partials live in their own buffer (ctx->scratch), so
    they cannot overwrite the staged B: one block row of 400 blocks (7
    segments) among 39 short ones, against the oracle."""
    rng = np.random.default_rng(77)
    mb, kb, bs, n = 40, 400, 32, 128
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.008)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(mb)]
    rows[5] = np.arange(kb, dtype=np.int32)
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1] * bs * bs).astype(np.float32)
    Bd = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    B = np.ascontiguousarray(Bd.T)
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    C = torch.full((mb * bs, n), float("nan"), device=device)
    _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=kb * bs, order_b=1, C=C,
                 ldc=n)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, Bd, n, 0)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F32, "segments + staged col-major B")


@pytest.mark.parametrize("layout", ["row", "col"])
@pytest.mark.parametrize("n", [8, 100])
def test_segments_long_rows_shallow_grid(oracle, device, layout, n):
    """512 block rows of ~130 blocks (2^16 blocks or more): a shallow grid. Row-major
    C splits the rows into segments summed by seg_fixup_kernel (each row past twice
    the mean load per slot); column-major C (transB = 1 with column-major C is
    test_bsrmm.cu:58's call) runs them longest first. Both layouts, the 64-column
    tile (n = 8) and the 128-column one, alpha / beta on the column-major one;
    against the f64 oracle, and the same bits on a second call. (Round 6 tried
    splitting every row of such grids, column-major C included: slower on the
    reference sweep at every fill, profiles/r06/ab_seg_shallow.log.)"""
    ops = _ops()
    rng = np.random.default_rng(5150 + n)
    mb, kb, bs = 512, 400, 32
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.33)
    assert rp[-1] >= 1 << 16
    m, k = mb * bs, kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = (1.0, 0.0) if layout == "row" else (0.5, -1.5)

    def run():
        if layout == "row":
            drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
            dC = torch.full((m * n,), float("nan"), device=device)
            ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n)
            torch.cuda.synchronize()
            return dC.cpu().numpy().reshape(m, n)
        drp, dci, dv, dB, dC = _dev(rp, ci, v, B.reshape(-1), np.ascontiguousarray(C0.T).reshape(-1))
        ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=m,
                  order_c=ops.ORDER_COL, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        return dC.cpu().numpy().reshape(n, m).T

    got = run()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    ref = alpha * ref + (beta * C0.astype(np.float64) if beta else 0.0)
    absd = abs(alpha) * absd + (abs(beta) * np.abs(C0.astype(np.float64)) if beta else 0.0)
    assert_normwise(got, ref, absd, TOL_F32, f"long rows, shallow grid, {layout} n={n}")
    assert np.array_equal(got.view(np.uint32), run().view(np.uint32))


@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("n", [1, 16, 33, 128, 512])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (0.5, 2.0)])
def test_bsrmm_mfma_shapes_alpha_beta(oracle, device, bs, n, alpha, beta):
    rng = np.random.default_rng(n + bs)
    mb, kb = 17, 21
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.3)
    Bd = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (mb * bs, n)).astype(np.float32)
    drp, dci, dv, dB, dC = _dev(rp, ci, v, Bd, C0)
    _ops().bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, alpha=alpha,
                 beta=beta)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, Bd, n, 0)
    assert_normwise(dC.cpu().numpy(), alpha * ref + beta * C0.astype(np.float64),
                    abs(alpha) * absd + abs(beta) * np.abs(C0), TOL_F32,
                    f"bs={bs} n={n} a={alpha} b={beta}")


@pytest.mark.parametrize("n", [16, 64, 128, 512])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("ob", [0, 1])
def test_bsrmm_f16(oracle, device, n, direction, ob):
    """fp16 A/B, fp32 accumulate: compared with the exact (f64) product of the
    same fp16 values; odd block counts exercise the half-empty MFMA pair."""
    rng = np.random.default_rng(n * 3 + direction)
    mb, kb, bs = 19, 25, 16
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.27, empty_rows=(0,))
    v16 = v.astype(np.float16)
    Bd = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float16)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    ldb = n if ob == 0 else kb * bs
    drp, dci, dv, dB = _dev(rp, ci, v16, B.reshape(-1))
    C = torch.empty((mb * bs, n), dtype=torch.float32, device=device)
    _ops().bsrmm_f16(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, order_b=ob, C=C,
                     ldc=n, direction=direction)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, direction, mb, n, bs, rp, ci, v16, Bd, n, 0, half=True)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F16_ACC, f"f16 n={n}")


@pytest.mark.parametrize("n", [136, 264, 392])
@pytest.mark.parametrize("oc", [0, 1])
@pytest.mark.parametrize("ob", [0, 1])
@pytest.mark.parametrize("cpad", [4, 1])
def test_bsrmm_f16_column_stream_shapes(oracle, device, n, oc, ob, cpad):
    """The shipped fp16 column streams (n >= 128) on the paths the defaults
    take besides n % 256 == 0: a ragged last column tile (n = 136, 264, 392:
    the clamped row offsets and the tail column guard), ldb > n, column-major
    C (the LDS-tile epilogue), alpha / beta != (1, 0) (the beta epilogue), and
    a column-major B staged row-major through the workspace; rows longer than
    one 64-block chunk and an empty block row. cpad = 1 makes ldc odd, so the
    row-major LDS-tile epilogue takes its per-element store path."""
    rng = np.random.default_rng(n * 7 + 2 * oc + ob)
    mb, kb, bs = 23, 90, 16
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.8, empty_rows=(4,))
    v16 = v.astype(np.float16)
    Bd = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float16)
    if ob == 0:
        ldb = n + 8
        Bm = np.zeros((kb * bs, ldb), np.float16)
        Bm[:, :n] = Bd
    else:
        ldb = kb * bs + 8
        Bm = np.zeros((n, ldb), np.float16)
        Bm[:, :kb * bs] = Bd.T
    m = mb * bs
    alpha, beta = 0.5, 1.5
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    ldc = n + cpad if oc == 0 else m + cpad
    Cm = np.zeros((m, ldc) if oc == 0 else (n, ldc), np.float32)
    if oc == 0:
        Cm[:, :n] = C0
    else:
        Cm[:, :m] = C0.T
    drp, dci, dv, dB, dC = _dev(rp, ci, v16, Bm.reshape(-1), Cm.reshape(-1))
    _ops().bsrmm_f16(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, order_b=ob, C=dC,
                     ldc=ldc, order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape(Cm.shape)
    got = got[:, :n] if oc == 0 else got[:, :m].T
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v16, Bd, n, 0, half=True)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(got, ref, absd, TOL_F16_ACC, f"f16 column stream n={n} oc={oc} ob={ob}")
    # the padding columns of C are untouched
    pad = dC.cpu().numpy().reshape(Cm.shape)[:, n:] if oc == 0 else \
        dC.cpu().numpy().reshape(Cm.shape)[:, m:]
    assert np.array_equal(pad, Cm[:, n:] if oc == 0 else Cm[:, m:])


def test_csr_vs_bsr_differential(oracle, device):
    """check_result.cu:103-116,233-246: csrmm2(T) vs bsrmm(T) after csr2bsr,
    m = 32768, p = 0.01, bs = 4, K = 64, B = +-0.5 alternating, eps 1e-4."""
    from spmm_hip import prep
    prep.rng_seed(1234)
    m, bs, K = 2 << 14, 4, 64
    rp, ci, v = prep.random_csr(m, m, 0.01)
    brp, bci, bval = prep.csr2bsr(m, m, rp, ci, v, bs)
    B = np.where(np.arange(m * K) % 2 == 0, 0.5, -0.5).astype(np.float32)
    drp, dci, dv, dB, dbrp, dbci, dbval = _dev(rp, ci, v, B, brp, bci, bval)
    C1 = torch.empty((m, K), device=device)
    C2 = torch.empty((m, K), device=device)
    ops = _ops()
    ops.csrmm(drp, dci, dv, dB, n=K, k=m, ldb=K, C=C1, ldc=K)
    ops.bsrmm(dbrp, dbci, dbval, dB, mb=m // bs, kb=m // bs, n=K, bs=bs, ldb=K, C=C2, ldc=K)
    torch.cuda.synchronize()
    assert float((C1 - C2).abs().max()) < 1e-4


@pytest.mark.parametrize("bs,density", [(16, 0.05), (32, 1.0 / 32), (32, 0.0), (8, 0.3)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (0.5, 1.5)])
def test_hybrid_divide_spmm(oracle, device, bs, density, alpha, beta):
    """divide.cu:348-373: BSR part (fill >= density) on MFMA + CSR remainder,
    one C; equals the plain CSR product of the whole matrix."""
    from spmm_hip import prep
    n, K = 700, 96
    rp, ci = prep.community_csr(n, 40.0, 48, 160, 0.9, 3)
    v = np.random.default_rng(4).uniform(-1, 1, ci.size).astype(np.float32)
    parts = prep.divide(n, rp, ci, v, bs, density)
    nb = (n + bs - 1) // bs
    Bp = np.zeros((nb * bs, K), np.float32)
    Bp[:n] = np.random.default_rng(5).uniform(-1, 1, (n, K))
    C0 = np.random.default_rng(6).uniform(-1, 1, (nb * bs, K)).astype(np.float32)
    d = _dev(*parts, Bp, C0)
    _ops().hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), d[6], m=n, n=K, k=n, bs=bs, ldb=K,
                        C=d[7], ldc=K, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, Bp, K, 0)
    got = d[7].cpu().numpy()[:n]
    assert_normwise(got, alpha * ref + beta * C0[:n].astype(np.float64),
                    abs(alpha) * absd + abs(beta) * np.abs(C0[:n]), TOL_F32,
                    f"hybrid bs={bs} density={density}")


@pytest.mark.parametrize("n,K", [(700, 96), (1000, 4), (963, 132), (2048, 256)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (0.5, 1.5)])
def test_hybrid_fused_vs_two_launch(oracle, device, n, K, alpha, beta):
    """The fused bs = 32 hybrid (SPMM_HYBRID_FUSED: one launch, MFMA part +
    per-block-row CSR remainder) against the oracle, and against the
    two-launch form (SPMM_HYBRID_TWO_LAUNCH): identical on every row the CSR kernel keeps in one wave.
    Hub rows give remainders far longer than the 32-entry batch, sparse rows
    give block rows with no dense block at all."""
    from spmm_hip import prep
    from spmm_hip._lib import (CSR_NT_STREAMS, CSR_SEQUENTIAL_ROWS, HYBRID_FUSED,
                               HYBRID_TWO_LAUNCH)
    rp, ci = prep.community_csr(n, 30.0, 48, 160, 0.9, 7)
    rng = np.random.default_rng(8)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(n)]
    rows[1] = np.arange(0, n, 2)                      # hub: long remainder
    rows[n // 2] = np.sort(rng.choice(n, n // 3, replace=False))
    for i in range(n - 40, n):                        # tail rows: remainder only
        rows[i] = np.sort(rng.choice(n, 3, replace=False))
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    parts = prep.divide(n, rp, ci, v, 32, 0.1)
    assert parts[4].size > 0 and parts[1].size > 0
    nb = (n + 31) // 32
    Bp = np.zeros((nb * 32, K), np.float32)
    Bp[:n] = rng.uniform(-1, 1, (n, K))
    C0 = rng.uniform(-1, 1, (nb * 32, K)).astype(np.float32)
    d = _dev(*parts, Bp)
    ops = _ops()
    outs = []
    for flags in (HYBRID_FUSED, HYBRID_TWO_LAUNCH):
        h = ops.Handle()
        h.set_hybrid_options(flags)
        # the small-K lane-group CSR kernel folds partial sums: compare
        # against the sequential-row kernel
        h.set_csr_options(CSR_NT_STREAMS | CSR_SEQUENTIAL_ROWS)
        C = torch.from_numpy(C0.copy()).cuda()
        ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), d[6], m=n, n=K, k=n, bs=32, ldb=K, C=C,
                         ldc=K, alpha=alpha, beta=beta, handle=h)
        torch.cuda.synchronize()
        outs.append(C.cpu().numpy())
        h.close()
    fused, two = outs
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, Bp, K, 0)
    assert_normwise(fused[:n], alpha * ref + beta * C0[:n].astype(np.float64),
                    abs(alpha) * absd + abs(beta) * np.abs(C0[:n]), TOL_F32, "fused hybrid")
    same = np.mean(np.all(fused[:n] == two[:n], axis=1))
    assert same > 0.9, f"only {same:.3f} of rows identical to the two-launch form"
    # padding rows (n .. nb*32): the BSR epilogue of an empty tail
    np.testing.assert_allclose(fused[n:], two[n:], rtol=0, atol=0)


@pytest.mark.parametrize("form", ["fused", "two_launch"])
def test_hybrid_split_bf16_alpha_beta_and_inf(oracle, device, form):
    """The split-bf16 epilogues with alpha != 1 and beta != 0 (C read), both
    launch forms; and an Inf in a dense block propagates as in fp32 (the
    split keeps Inf in the high part instead of making Inf - Inf = NaN)."""
    from spmm_hip import prep
    from spmm_hip._lib import HYBRID_FUSED, HYBRID_SPLIT_BF16, HYBRID_TWO_LAUNCH
    ops = _ops()
    rng = np.random.default_rng(31)
    n, K, bs = 1000, 128, 32
    rp, ci, v = _rand_csr_blocky(rng, n, bs)
    parts = prep.divide(n, rp, ci, v, bs, 0.25)
    mb = (n + bs - 1) // bs
    B = rng.uniform(-1, 1, (mb * bs, K)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (mb * bs, K)).astype(np.float32)
    alpha, beta = 0.75, -1.25
    flags = HYBRID_SPLIT_BF16 | (HYBRID_FUSED if form == "fused" else HYBRID_TWO_LAUNCH)
    h = ops.Handle()
    h.set_hybrid_options(flags)
    d = _dev(*parts)
    dB, dC = _dev(B, C0)
    ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), dB, m=n, n=K, k=n, bs=bs, ldb=K, C=dC, ldc=K,
                     alpha=alpha, beta=beta, handle=h)
    torch.cuda.synchronize()
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, B[:n], K, 0)
    want = alpha * ref + beta * C0[:n].astype(np.float64)
    bound = abs(alpha) * absd + abs(beta) * np.abs(C0[:n])
    assert_normwise(dC.cpu().numpy()[:n], want, bound, TOL_F32, f"split-bf16 {form} alpha/beta")
    # Inf in one dense-block value: rows meeting it become +-Inf, none NaN
    bval = parts[5].copy()
    assert bval.size
    bval[0] = np.inf
    d2 = _dev(parts[0], parts[1], parts[2], parts[3], parts[4], bval)
    dC2 = torch.empty((mb * bs, K), dtype=torch.float32, device=device)
    ops.hybrid_csrmm(tuple(d2[0:3]), tuple(d2[3:6]), dB, m=n, n=K, k=n, bs=bs, ldb=K, C=dC2,
                     ldc=K, handle=h)
    torch.cuda.synchronize()
    got = dC2.cpu().numpy()
    r0 = 0  # block 0 of block row 0, entry (0, 0): row 0, column 32 * bci[0]
    assert np.isinf(got[r0]).all() and not np.isnan(got[:n]).any()
    h.close()


def _rand_csr_blocky(rng, n, bs):
    """A CSR with dense diagonal-ish blocks plus scattered entries (so divide
    keeps a BSR part and a CSR remainder)."""
    rows = []
    for r in range(n):
        b = r // bs
        dense = b * bs + rng.choice(bs, 20, replace=False)
        far = rng.choice(n, 3, replace=False)
        rows.append(np.unique(np.concatenate([dense[dense < n], far])))
    rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    return rp, ci, v


@pytest.mark.parametrize("form", ["fused", "two_launch"])
@pytest.mark.parametrize("n,K", [(1000, 128), (963, 132)])
def test_hybrid_split_bf16(oracle, device, form, n, K):
    """SPMM_HYBRID_SPLIT_BF16: the dense-block part's fp32 products as six bf16
    MFMA products of an exact three-way split. Held to the fp32 bar element by
    element (|err| <= 1e-5 |A||B|) on values spread over six decades, and
    within 2^-18 |A||B| of the fp32-MFMA form."""
    from spmm_hip import prep
    from spmm_hip._lib import HYBRID_FUSED, HYBRID_SPLIT_BF16, HYBRID_TWO_LAUNCH
    rp, ci = prep.community_csr(n, 40.0, 48, 160, 0.95, 11)
    rng = np.random.default_rng(12)
    v = (rng.uniform(-1, 1, ci.size) * 10.0 ** rng.uniform(-3, 3, ci.size)).astype(np.float32)
    parts = prep.divide(n, rp, ci, v, 32, 0.05)
    assert parts[4].size > 0 and parts[1].size > 0
    nb = (n + 31) // 32
    Bp = np.zeros((nb * 32, K), np.float32)
    Bp[:n] = rng.uniform(-1, 1, (n, K)) * 10.0 ** rng.uniform(-3, 3, (n, K))
    d = _dev(*parts, Bp)
    ops = _ops()
    base = HYBRID_FUSED if form == "fused" else HYBRID_TWO_LAUNCH
    outs = []
    for flags in (base | HYBRID_SPLIT_BF16, base):
        h = ops.Handle()
        h.set_hybrid_options(flags)
        C = torch.empty((nb * 32, K), device=device)
        ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), d[6], m=n, n=K, k=n, bs=32, ldb=K, C=C,
                         ldc=K, handle=h)
        torch.cuda.synchronize()
        outs.append(C.cpu().numpy()[:n].astype(np.float64))
        h.close()
    split, plain = outs
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, Bp, K, 0)
    err = np.abs(split - ref)
    assert np.all(err <= TOL_F32 * absd + 1e-30), \
        f"split-bf16 {form}: max err / |A||B| {np.max(err / (absd + 1e-30)):.3g}"
    assert np.all(np.abs(split - plain) <= 2.0 ** -18 * absd + 1e-30)


def test_bsr_status_codes(device):
    """rocsparse_bsrmm.h:109-176 argument checks."""
    from spmm_hip._lib import (INVALID_VALUE, MATRIX_TYPE_NOT_SUPPORTED, NOT_INITIALIZED,
                               SUCCESS, lib)
    L = lib()
    h = _ops().default_handle()
    d = ctypes.c_void_p()
    L.spmm_create_mat_descr(ctypes.byref(d))
    one = ctypes.c_float(1.0)
    args = lambda **kw: dict(dict(handle=h.raw, dir=0, ta=0, tb=0, mb=2, n=2, kb=3, nnzb=4,
                                  descr=d, bs=2, ldb=6, ldc=4), **kw)

    def call(a, C=None):
        return L.spmm_sbsrmm(a["handle"], a["dir"], a["ta"], a["tb"], a["mb"], a["n"], a["kb"],
                             a["nnzb"], ctypes.byref(one), a["descr"], C, C, C, a["bs"], C,
                             a["ldb"], ctypes.byref(one), C, a["ldc"])

    assert call(args(handle=None)) == NOT_INITIALIZED
    assert call(args(descr=None)) == INVALID_VALUE
    assert call(args(ta=1)) == MATRIX_TYPE_NOT_SUPPORTED
    assert call(args(tb=2)) == MATRIX_TYPE_NOT_SUPPORTED
    assert call(args(mb=-1)) == INVALID_VALUE
    assert call(args(bs=0)) == INVALID_VALUE
    assert call(args(nnzb=0)) == SUCCESS  # quick return, nothing touched
    assert call(args()) == INVALID_VALUE  # null pointers
    L.spmm_destroy_mat_descr(d)


@pytest.mark.parametrize("bs,dtype", [(32, "f32"), (16, "f32"), (16, "f16")])
@pytest.mark.parametrize("n", [8, 96, 264, 520])
@pytest.mark.parametrize("oc", [0, 1])
def test_lds_staged_kernels(oracle, device, bs, dtype, n, oc):
    """The LDS-staged MFMA kernels (ROW blocks, row-major B): several column
    tiles with a partial last one, ldb > n, empty block rows, one-block rows
    (the clamped copy tail), long rows (cursor refills past 64 blocks), and
    both C orders, with alpha/beta."""
    rng = np.random.default_rng(n * 7 + bs + oc)
    mb, kb = 23, 90
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.25, empty_rows=(0, 5))
    # row 7: one block; row 9: every block column (90 > 64 blocks)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(mb)]
    rows[7] = np.array([kb - 1])
    rows[9] = np.arange(kb)
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1] * bs * bs).astype(np.float32)
    ldb = n + 8
    Bfull = rng.uniform(-1, 1, (kb * bs, ldb)).astype(np.float32)
    m = mb * bs
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = 0.75, -0.5
    if dtype == "f16":
        v, Bfull = v.astype(np.float16), Bfull.astype(np.float16)
    ldc = n if oc == 0 else m
    Cinit = C0 if oc == 0 else np.ascontiguousarray(C0.T)
    drp, dci, dv, dB, dC = _dev(rp, ci, v, Bfull.reshape(-1), Cinit.reshape(-1))
    fn = _ops().bsrmm if dtype == "f32" else _ops().bsrmm_f16
    fn(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, C=dC, ldc=ldc, order_c=oc,
       alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape(Cinit.shape)
    got = got if oc == 0 else got.T
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, Bfull[:, :n], n, 0,
                                 half=dtype == "f16")
    tol = TOL_F32 if dtype == "f32" else TOL_F16_ACC
    assert_normwise(got, alpha * ref + beta * C0, abs(alpha) * absd + abs(beta) * np.abs(C0), tol,
                    f"lds bs={bs} {dtype} n={n} oc={oc}")


def _column_sparse_bsr(rng, mb, kb, bs, p):
    """BSR whose blocks are mostly empty columns, like csr2bsr output of a
    sparse graph: per block a random number of active columns (0 = an
    explicit all-zero block, 1 = a single-column block, up to bs), each
    active column holding a few nonzeros."""
    rp, ci, _ = _rand_bsr(rng, mb, kb, bs, p, empty_rows=(3,))
    nnzb = int(rp[-1])
    v = np.zeros((nnzb, bs, bs), np.float32)
    for b in range(nnzb):
        kind = b % 5
        ncols = {0: 0, 1: 1, 2: 2, 3: bs // 4, 4: bs}[kind]
        cols = rng.choice(bs, ncols, replace=False)
        for c in cols:
            rows = rng.random(bs) < 0.3
            rows[rng.integers(bs)] = True
            v[b, rows, c] = rng.uniform(-1, 1, int(rows.sum()))
    return rp, ci, v.reshape(-1)


@pytest.mark.parametrize("bs,dtype", [(32, "f32"), (16, "f32"), (16, "f16")])
@pytest.mark.parametrize("n", [64, 128, 264, 520])
@pytest.mark.parametrize("layout", ["row", "col"])
def test_column_sparse_blocks(oracle, device, bs, dtype, n, layout):
    _column_sparse_blocks(oracle, device, bs, dtype, n, layout)


@pytest.mark.parametrize("bs", [32, 64])
@pytest.mark.parametrize("n", [64, 36, 8])
@pytest.mark.parametrize("layout", ["row", "col"])
def test_narrow_tile_bit_exact(oracle, device, bs, n, layout):
    """n <= 64 runs the column stream's 64-column tile (bsr32_f32_cs2_kernel
    C64, bs 32 and the bs 64 sub-block stream; the reference sweeps dim 64,
    benchmark.py:5-8). Every column is the same MFMA chain as in the 128-column
    tile: C equals the first n columns of the n = 128 product on [B | B2] bit
    for bit, and the sequential fp32 oracle (rocsparse_bsrmm_template<float>'s
    order) bit for bit; both layouts, alpha / beta on the column-major one."""
    ops = _ops()
    rng = np.random.default_rng(640 + n + bs)
    mb, kb = 19, 40
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.35)
    m, k = mb * bs, kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    B2 = np.concatenate([B, rng.uniform(-1, 1, (k, 128 - n)).astype(np.float32)], axis=1)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = (1.0, 0.0) if layout == "row" else (0.5, -1.5)

    def run(Bh, nn, c0):
        ldb = nn
        if layout == "row":
            drp, dci, dv, dB = _dev(rp, ci, v, Bh.reshape(-1))
            dC = torch.full((m * nn,), float("nan"), device=device)
            ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=nn, bs=bs, ldb=ldb, C=dC, ldc=nn)
            torch.cuda.synchronize()
            return dC.cpu().numpy().reshape(m, nn)
        drp, dci, dv, dB, dC = _dev(rp, ci, v, np.ascontiguousarray(Bh.T).reshape(-1),
                                    np.ascontiguousarray(c0.T).reshape(-1))
        ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=nn, bs=bs, ldb=k, order_b=ops.ORDER_COL,
                  C=dC, ldc=m, order_c=ops.ORDER_COL, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        return dC.cpu().numpy().reshape(nn, m).T

    got = run(B, n, C0)
    C0w = np.concatenate([C0, np.zeros((m, 128 - n), np.float32)], axis=1)
    wide = run(B2, 128, C0w)
    assert np.array_equal(got, wide[:, :n]), "the 64-column tile differs from the 128-column one"
    ref = oracle_bsrmm_f32(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0, alpha=alpha, beta=beta,
                           C=C0.reshape(-1) if layout == "col" else None).reshape(m, n)
    ref64, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    if layout == "col":
        ref64 = alpha * ref64 + beta * C0.astype(np.float64)
        absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(got, ref64, absd, TOL_F32, f"narrow tile bs={bs} n={n} {layout}")
    if layout == "row":
        assert np.array_equal(got, ref), "not the sequential fp32 chain"


def _column_sparse_blocks(oracle, device, bs, dtype, n, layout):
    """Blocks with empty columns (the column-masked kernels fetch only the B
    rows of nonzero A columns and skip MFMA steps of empty ones): explicit
    zero blocks, single-column blocks, quarter-full and full blocks, empty
    block rows, long rows. Then the same with inf / NaN in B rows that only
    empty A columns meet: those entries act as structural zeros (the CSR
    semantics of the same matrix), so C stays finite and equal to the
    product with those rows zeroed. layout "col" is cusparseSbsrmm's
    transB = N form (column-major B and C, alpha / beta), which the library
    stages through its workspace onto the same kernels."""
    rng = np.random.default_rng(n + bs)
    mb, kb = 21, 80
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.3)
    ldb = n
    B = rng.uniform(-1, 1, (kb * bs, ldb)).astype(np.float32)
    if dtype == "f16":
        v, B = v.astype(np.float16), B.astype(np.float16)
    fn = _ops().bsrmm if dtype == "f32" else _ops().bsrmm_f16
    m = mb * bs
    tol = TOL_F32 if dtype == "f32" else TOL_F16_ACC

    ops = _ops()
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = (1.0, 0.0) if layout == "row" else (0.5, -1.5)

    def run(Bh):
        if layout == "row":  # row-major B and C, beta = 0: C starts as NaN
            drp, dci, dv, dB = _dev(rp, ci, v, Bh.reshape(-1))
            dC = torch.full((m * n,), float("nan"), device=device)
            fn(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldb, C=dC, ldc=n)
            torch.cuda.synchronize()
            return dC.cpu().numpy().reshape(m, n)
        # cusparseSbsrmm transB = N: B and C column-major (staged through the workspace)
        drp, dci, dv, dB, dC = _dev(rp, ci, v, np.ascontiguousarray(Bh.T).reshape(-1),
                                    np.ascontiguousarray(C0.T).reshape(-1))
        fn(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=kb * bs, order_b=ops.ORDER_COL, C=dC,
           ldc=m, order_c=ops.ORDER_COL, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        return dC.cpu().numpy().reshape(n, m).T

    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, ldb, 0,
                                 half=dtype == "f16")
    c0 = 0.0 if layout == "row" else C0.astype(np.float64)
    ref = alpha * ref + beta * c0
    absd = abs(alpha) * absd + abs(beta) * np.abs(c0)
    what = f"column-sparse bs={bs} {dtype} n={n} {layout}"
    assert_normwise(run(B), ref, absd, tol, what)
    # B rows that no nonzero of A meets
    vb = v.reshape(-1, bs, bs).astype(np.float32)
    used = np.zeros(kb * bs, bool)
    for br in range(mb):
        for k in range(rp[br], rp[br + 1]):
            used[ci[k] * bs + np.nonzero(np.any(vb[k] != 0, axis=0))[0]] = True
    unused = np.nonzero(~used)[0]
    assert unused.size > 0
    Bbad = B.copy()
    Bbad[unused[0::2]] = np.inf
    Bbad[unused[1::2]] = np.nan
    got = run(Bbad)
    assert np.isfinite(got).all(), "explicit zeros must not turn inf / NaN of B into NaN"
    assert_normwise(got, ref, absd, tol, what + ", non-finite B")


@pytest.mark.parametrize("bs,dtype", [(32, "f32"), (16, "f32"), (16, "f16"), (8, "f32"),
                                      (64, "f32")])
@pytest.mark.parametrize("layout", ["row", "col"])
def test_dense_block_product_option(oracle, device, bs, dtype, layout):
    """SPMM_BSR_DENSE_BLOCK_PRODUCT (spmm_set_bsr_options): cusparseSbsrmm's
    dense-block semantics. inf / NaN in B rows that only explicit zeros of
    stored blocks meet give NaN in every row of those block rows (0 * inf),
    exactly where the f64 dense-block oracle has them; every other element
    matches the oracle within the bar. The default handle on the same inputs
    keeps them finite (column-granular contract, test_column_sparse_blocks)."""
    from spmm_hip._lib import BSR_DENSE_BLOCK_PRODUCT
    ops = _ops()
    rng = np.random.default_rng(7 * bs + (layout == "col"))
    mb, kb, n = 13, 40, 136
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.3)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    vb = v.reshape(-1, bs, bs)
    used = np.zeros(kb * bs, bool)
    stored = np.zeros(kb * bs, bool)
    for k in range(rp[-1]):
        used[ci[k] * bs + np.nonzero(np.any(vb[k] != 0, axis=0))[0]] = True
        stored[ci[k] * bs: ci[k] * bs + bs] = True
    cand = np.nonzero(stored & ~used)[0]
    assert cand.size >= 2
    B[cand[0]] = np.inf
    B[cand[1]] = np.nan
    if dtype == "f16":
        v, B = v.astype(np.float16), B.astype(np.float16)
    fn = ops.bsrmm if dtype == "f32" else ops.bsrmm_f16
    m = mb * bs
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0, half=dtype == "f16")
    for flags in (BSR_DENSE_BLOCK_PRODUCT, 0):
        h = ops.Handle()
        h.set_bsr_options(flags)
        if layout == "row":
            drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
            dC = torch.empty((m * n,), device=device)
            fn(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, handle=h)
            torch.cuda.synchronize()
            got = dC.cpu().numpy().reshape(m, n)
        else:
            drp, dci, dv, dB = _dev(rp, ci, v, np.ascontiguousarray(B.T).reshape(-1))
            dC = torch.empty((n * m,), device=device)
            fn(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=kb * bs, order_b=ops.ORDER_COL,
               C=dC, ldc=m, order_c=ops.ORDER_COL, handle=h)
            torch.cuda.synchronize()
            got = dC.cpu().numpy().reshape(n, m).T
        h.close()
        what = f"bs={bs} {dtype} {layout} flags={flags}"
        if flags:
            assert np.isnan(ref).any()
            assert np.array_equal(np.isnan(got), np.isnan(ref)), what + ": NaN pattern"
            fin = ~np.isnan(ref)
            assert_normwise(got[fin], ref[fin], absd[fin], TOL_F32 if dtype == "f32" else
                            TOL_F16_ACC, what)
        else:  # the column streams, column-masked and lane-group kernels skip empty columns
            assert np.isfinite(got).all(), what + ": default contract keeps C finite"


def _masks_np(v, bs=32):
    """Column masks of row-major blocks as the analysis defines them (bit c: a
    value other than +-0 in column c; NaN and inf count)."""
    vb = v.reshape(-1, bs, bs)
    nz = (vb.view(np.uint32) & 0x7fffffff) != 0
    cols = nz.any(axis=1)  # [nnzb, bs]
    return (cols.astype(np.uint64) << np.arange(bs, dtype=np.uint64)).sum(axis=1).astype(np.uint32)


@pytest.mark.parametrize("direction", [0, 1])
def test_bsr32_analysis(device, direction):
    """spmm_bsr32_analysis_f32: the column masks (explicit zero blocks, -0.0,
    NaN and inf entries included) and, for ROW blocks, the column-major copy."""
    rng = np.random.default_rng(5 + direction)
    rp, ci, v = _column_sparse_bsr(rng, 17, 40, 32, 0.4)
    vb = v.reshape(-1, 32, 32).copy()
    nnzb = vb.shape[0]
    vb[1, 3, 7] = -0.0
    vb[2, 0, 31] = np.nan
    vb[4, 31, 0] = np.inf
    v = vb.reshape(-1)
    src = v if direction == 0 else np.ascontiguousarray(vb.transpose(0, 2, 1)).reshape(-1)
    (dv,) = _dev(src)
    masks, vcol = _ops().bsr32_analysis(dv, nnzb=nnzb, direction=direction)
    torch.cuda.synchronize()
    want = _masks_np(v)
    got = masks.cpu().numpy()[:nnzb].view(np.uint32)
    assert np.array_equal(got, want)
    colmajor = np.ascontiguousarray(vb.transpose(0, 2, 1)).reshape(-1)
    assert np.array_equal(vcol.cpu().numpy()[:nnzb * 1024].view(np.uint32),
                          colmajor.view(np.uint32))


@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("n", [96, 136, 130])
@pytest.mark.parametrize("direction", [0, 1])
def test_bsrmm_analysed(oracle, device, orders, n, direction):
    """spmm_bsrmm_analysed_f32 against the fp64 oracle: column-sparse blocks,
    an empty block row and one of 300 blocks (several 64-block chunks, and
    segments on this shallow grid), alpha / beta, every B / C order; n = 130
    (n % 4 != 0) takes the COLUMN-direction fallback kernels on the same
    analysis. Then inf / NaN in B rows that only empty columns meet: C stays
    finite, as with the other column streams."""
    ob, oc = orders
    rng = np.random.default_rng(n + 10 * ob + 100 * oc + direction)
    mb, kb, bs = 23, 320, 32
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.1)
    # block row 5: 300 blocks
    rows = [ci[rp[i]:rp[i + 1]] for i in range(mb)]
    vals = [v.reshape(-1, bs * bs)[rp[i]:rp[i + 1]] for i in range(mb)]
    rows[5] = np.sort(rng.choice(kb, 300, replace=False)).astype(np.int32)
    _, _, extra = _column_sparse_bsr(rng, 1, 300, bs, 1.0)
    vals[5] = extra.reshape(-1, bs * bs)[:300]
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = np.concatenate(vals).reshape(-1).astype(np.float32)
    nnzb = ci.size
    K, m = kb * bs, mb * bs
    Bd = rng.uniform(-1, 1, (K, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = 0.5, -1.5
    ops = _ops()
    src = v if direction == 0 else np.ascontiguousarray(
        v.reshape(-1, bs, bs).transpose(0, 2, 1)).reshape(-1)
    drp, dci, dv = _dev(rp, ci, src)
    masks, vcol = ops.bsr32_analysis(dv, nnzb=nnzb, direction=direction)

    def run(Bh):
        B = Bh if ob == 0 else np.ascontiguousarray(Bh.T)
        Cm = C0 if oc == 0 else np.ascontiguousarray(C0.T)
        dB, dC = _dev(B.reshape(-1), Cm.reshape(-1))
        ops.bsrmm_analysed(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n,
                           ldb=n if ob == 0 else K, order_b=ob, C=dC, ldc=n if oc == 0 else m,
                           order_c=oc, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        got = dC.cpu().numpy().reshape((m, n) if oc == 0 else (n, m))
        return got if oc == 0 else got.T

    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, Bd, n, 0)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    what = f"analysed n={n} orders={orders} dir={direction}"
    assert_normwise(run(Bd), ref, absd, TOL_F32, what)
    if n % 4:
        return  # the fallback kernels compute the dense block product
    vb = v.reshape(-1, bs, bs)
    used = np.zeros(K, bool)
    for br in range(mb):
        for k in range(rp[br], rp[br + 1]):
            used[ci[k] * bs + np.nonzero(np.any(vb[k] != 0, axis=0))[0]] = True
    unused = np.nonzero(~used)[0]
    assert unused.size > 0
    Bbad = Bd.copy()
    Bbad[unused[0::2]] = np.inf
    Bbad[unused[1::2]] = np.nan
    got = run(Bbad)
    assert np.isfinite(got).all()
    assert_normwise(got, ref, absd, TOL_F32, what + ", non-finite B")


def test_bsrmm_analysed_matches_column_stream(device):
    """The analysed stream is the shipped bs 32 column stream with A read from
    the column-major copy: the same items in the same order, so the same
    result bit for bit (row-major B and C)."""
    rng = np.random.default_rng(77)
    mb, kb, bs, n = 40, 200, 32, 256
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.15)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    ops = _ops()
    C1 = torch.empty((mb * bs, n), device=device)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=n)
    masks, vcol = ops.bsr32_analysis(dv, nnzb=ci.size)
    C2 = torch.empty((mb * bs, n), device=device)
    ops.bsrmm_analysed(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=C2, ldc=n)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)


def test_bsr32_analysis_argument_checks(device):
    """Status codes of the analysis entries (the reference's INVALID_VALUE /
    quick-return conventions, rocsparse_bsrmm.h:110-176)."""
    from spmm_hip._lib import lib
    h = _ops().default_handle()
    v = torch.zeros(2048, device=device)
    m = torch.zeros(2, dtype=torch.int32, device=device)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    L = lib()
    assert L.spmm_bsr32_analysis_f32(h.raw, 5, 2, P(v), P(m), P(v)) == 3      # bad dir
    assert L.spmm_bsr32_analysis_f32(h.raw, 0, -1, P(v), P(m), P(v)) == 3     # nnzb < 0
    assert L.spmm_bsr32_analysis_f32(h.raw, 0, 2, P(v), P(m), None) == 3      # ROW needs valCol
    assert L.spmm_bsr32_analysis_f32(h.raw, 1, 2, P(v), P(m), None) == 0      # COLUMN does not
    assert L.spmm_bsr32_analysis_f32(h.raw, 0, 0, None, None, None) == 0      # quick return
    rp = torch.tensor([0, 2], dtype=torch.int32, device=device)
    ci = torch.tensor([0, 1], dtype=torch.int32, device=device)
    B = torch.zeros(64 * 8, device=device)
    C = torch.full((32 * 8,), 3.0, device=device)
    args = (h.raw, 1, 2, 8, 2, 1.0, P(rp), P(ci), P(v))
    assert L.spmm_bsrmm_analysed_f32(*args, None, P(B), 8, 0, 0.0, P(C), 8, 0) == 3  # masks
    assert L.spmm_bsrmm_analysed_f32(*args, P(m), P(B), 4, 0, 0.0, P(C), 8, 0) == 3  # ldb < n
    assert L.spmm_bsrmm_analysed_f32(h.raw, 0, 2, 8, 2, 1.0, None, None, None, None, None, 8, 0,
                                     0.0, None, 8, 0) == 0                            # quick
    torch.cuda.synchronize()
    assert torch.all(C == 3.0)


def _masks16_np(v16):
    vb = v16.reshape(-1, 16, 16)
    nz = (vb.view(np.uint16) & 0x7fff) != 0
    cols = nz.any(axis=1)
    return (cols.astype(np.uint32) << np.arange(16, dtype=np.uint32)).sum(axis=1).astype(np.uint32)


@pytest.mark.parametrize("direction", [0, 1])
def test_bsr16_analysis(device, direction):
    """spmm_bsr16_analysis_f16: masks (-0.0, NaN, inf included) and the
    column-major fp16 copy of ROW blocks."""
    rng = np.random.default_rng(15 + direction)
    rp, ci, v = _column_sparse_bsr(rng, 19, 50, 16, 0.4)
    vb = v.astype(np.float16).reshape(-1, 16, 16).copy()
    nnzb = vb.shape[0]
    vb[1, 3, 7] = -0.0
    vb[2, 0, 15] = np.nan
    vb[4, 15, 0] = np.inf
    src = vb.reshape(-1) if direction == 0 else np.ascontiguousarray(
        vb.transpose(0, 2, 1)).reshape(-1)
    (dv,) = _dev(src)
    masks, vcol = _ops().bsr16_analysis(dv, nnzb=nnzb, direction=direction)
    torch.cuda.synchronize()
    assert np.array_equal(masks.cpu().numpy()[:nnzb].view(np.uint32), _masks16_np(vb))
    colmajor = np.ascontiguousarray(vb.transpose(0, 2, 1)).reshape(-1)
    assert np.array_equal(vcol.cpu().numpy()[:nnzb * 256].view(np.uint16),
                          colmajor.view(np.uint16))


@pytest.mark.parametrize("orders", [(0, 0), (1, 1), (0, 1)])
@pytest.mark.parametrize("n", [128, 264, 512, 120])
@pytest.mark.parametrize("direction", [0, 1])
def test_bsrmm_analysed_f16(oracle, device, orders, n, direction):
    """spmm_bsrmm_analysed_f16 against the fp64 oracle (fp16 inputs): column-
    sparse blocks, an empty block row, one of 300 blocks (several 64-block
    chunks), alpha / beta, B / C orders; n = 120 (< 128) takes the COLUMN-
    direction fallback. Then inf / NaN in B rows only empty columns meet."""
    ob, oc = orders
    rng = np.random.default_rng(3 * n + 10 * ob + 100 * oc + direction)
    mb, kb, bs = 21, 320, 16
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.1)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(mb)]
    vals = [v.reshape(-1, bs * bs)[rp[i]:rp[i + 1]] for i in range(mb)]
    rows[5] = np.sort(rng.choice(kb, 300, replace=False)).astype(np.int32)
    _, _, extra = _column_sparse_bsr(rng, 1, 300, bs, 1.0)
    vals[5] = extra.reshape(-1, bs * bs)[:300]
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v16 = np.concatenate(vals).reshape(-1).astype(np.float16)
    nnzb = ci.size
    K, m = kb * bs, mb * bs
    Bd = rng.uniform(-1, 1, (K, n)).astype(np.float16)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = 0.5, -1.5
    ops = _ops()
    src = v16 if direction == 0 else np.ascontiguousarray(
        v16.reshape(-1, bs, bs).transpose(0, 2, 1)).reshape(-1)
    drp, dci, dv = _dev(rp, ci, src)
    masks, vcol = ops.bsr16_analysis(dv, nnzb=nnzb, direction=direction)

    def run(Bh):
        B = Bh if ob == 0 else np.ascontiguousarray(Bh.T)
        Cm = C0 if oc == 0 else np.ascontiguousarray(C0.T)
        dB, dC = _dev(B.reshape(-1), Cm.reshape(-1))
        ops.bsrmm_analysed_f16(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n,
                               ldb=n if ob == 0 else K, order_b=ob, C=dC,
                               ldc=n if oc == 0 else m, order_c=oc, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        got = dC.cpu().numpy().reshape((m, n) if oc == 0 else (n, m))
        return got if oc == 0 else got.T

    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v16, Bd, n, 0, half=True)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    what = f"analysed f16 n={n} orders={orders} dir={direction}"
    assert_normwise(run(Bd), ref, absd, TOL_F16_ACC, what)
    if n < 128:
        return  # the fallback kernels compute the dense block product
    vb = v16.reshape(-1, bs, bs)
    used = np.zeros(K, bool)
    for br in range(mb):
        for k in range(rp[br], rp[br + 1]):
            used[ci[k] * bs + np.nonzero(np.any(vb[k] != 0, axis=0))[0]] = True
    unused = np.nonzero(~used)[0]
    assert unused.size > 0
    Bbad = Bd.copy()
    Bbad[unused[0::2]] = np.inf
    Bbad[unused[1::2]] = np.nan
    got = run(Bbad)
    assert np.isfinite(got).all()
    assert_normwise(got, ref, absd, TOL_F16_ACC, what + ", non-finite B")


def test_bsrmm_analysed_f16_matches_column_stream(device):
    """Same items in the same order as the shipped fp16 column stream: the
    same result bit for bit."""
    rng = np.random.default_rng(78)
    mb, kb, bs, n = 40, 300, 16, 512
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.15)
    v16 = v.astype(np.float16)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float16)
    drp, dci, dv, dB = _dev(rp, ci, v16, B.reshape(-1))
    ops = _ops()
    C1 = torch.empty((mb * bs, n), device=device)
    ops.bsrmm_f16(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=n)
    masks, vcol = ops.bsr16_analysis(dv, nnzb=ci.size)
    C2 = torch.empty((mb * bs, n), device=device)
    ops.bsrmm_analysed_f16(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=C2, ldc=n)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)


@pytest.mark.parametrize("bs", [2, 4, 8])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("n", [64, 130, 256])
def test_small_bs_lane_group_bit_exact(oracle, device, bs, direction, n):
    """bs 2 / 4 / 8 (bsr_small_kernel): every output element is the oracle's
    sequential fp32 FMA chain (blocks in order, columns in order,
    oracle_bsrmm_f32 = rocsparse_bsrmm_template<float>'s order) bit for bit,
    long and empty block rows included; alpha / beta on a second call."""
    ops = _ops()
    rng = np.random.default_rng(100 * bs + 10 * direction + n % 7)
    mb, kb = 37, 300 // bs
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.25, empty_rows=(5,))
    vb = v.reshape(-1, bs, bs)  # about half the block columns empty (the zero-row gathers)
    for k in range(vb.shape[0]):
        dead = rng.random(bs) < 0.5
        if direction == 0:
            vb[k][:, dead] = 0.0
        else:
            vb[k][dead, :] = 0.0
    v = vb.reshape(-1)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    C = torch.full((mb * bs, n), float("nan"), device=device)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C, ldc=n, direction=direction)
    torch.cuda.synchronize()
    want = oracle_bsrmm_f32(oracle, direction, mb, n, bs, rp, ci, v, B, n, 0).reshape(mb * bs, n)
    got = C.cpu().numpy()
    assert (got == want).all(), f"bs {bs}: {int((got != want).sum())} elements differ"
    C0 = rng.uniform(-1, 1, (mb * bs, n)).astype(np.float32)
    dC = _dev(C0)[0]
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, alpha=0.5, beta=-2.0,
              direction=direction)
    torch.cuda.synchronize()
    want2 = oracle_bsrmm_f32(oracle, direction, mb, n, bs, rp, ci, v, B, n, 0, 0.5, -2.0, C0,
                             n, 0).reshape(mb * bs, n)
    assert (dC.cpu().numpy() == want2).all(), f"bs {bs}: alpha / beta epilogue"


def _grouped_handle():
    """A handle whose bs 2 / 4 / 8 products take the grouped MFMA stream at any size
    (SPMM_BSR_SMALL_GROUPED; by default only from 2^20 blocks)."""
    from spmm_hip._lib import BSR_SMALL_GROUPED
    h = _ops().Handle()
    h.set_bsr_options(BSR_SMALL_GROUPED)
    return h


def test_bsr_options_flags(device):
    """spmm_set_bsr_options takes SPMM_BSR_DENSE_BLOCK_PRODUCT and
    SPMM_BSR_SMALL_GROUPED, alone or together, and refuses any other bit."""
    from spmm_hip._lib import BSR_DENSE_BLOCK_PRODUCT, BSR_SMALL_GROUPED, SpmmError
    h = _ops().Handle()
    for f in (0, BSR_DENSE_BLOCK_PRODUCT, BSR_SMALL_GROUPED,
              BSR_DENSE_BLOCK_PRODUCT | BSR_SMALL_GROUPED):
        h.set_bsr_options(f)
    with pytest.raises(SpmmError):
        h.set_bsr_options(4)
    h.close()


def _grouped_small_bsr(rng, bs, mb, kb, sorted_cols=True):
    """Block rows in runs that share block columns (neighbouring rows of a
    community), power-law lengths from empty to past several merge batches,
    about half the columns of each block empty."""
    rows = []
    for br in range(mb):
        L = int(min(kb, rng.pareto(1.2) * 6)) if br % 7 != 3 else 0
        home = (br // 3) * 5 % kb
        near = (home + rng.integers(0, 24, L)) % kb
        far = rng.integers(0, kb, max(L // 3, 0))
        c = np.unique(np.concatenate([near, far]))[:L] if L else np.zeros(0, np.int64)
        if not sorted_cols:
            c = rng.permutation(c)
        rows.append(c)
    rp = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    vb = rng.uniform(-1, 1, (rp[-1], bs, bs)).astype(np.float32)
    for k in range(vb.shape[0]):
        vb[k][:, rng.random(bs) < 0.5] = 0.0
    return rp, ci, vb


@pytest.mark.parametrize("bs", [2, 4, 8])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("n,oc", [(128, 0), (384, 0), (64, 0), (256, 1)])
def test_small_bs_grouped_stream_bit_exact(oracle, device, bs, direction, n, oc):
    """bs 2 / 4 / 8 on the grouped MFMA stream (bsr_small_grp_kernel: 32 / bs
    block rows per wave walk the union of their block columns): every element
    is the oracle's sequential fp32 FMA chain bit for bit, over rows that span
    many merge batches, runs of rows sharing columns, empty rows, a last group
    cut short, several 128-column tiles and column-major C; alpha / beta."""
    ops = _ops()
    h = _grouped_handle()
    rng = np.random.default_rng(1000 * bs + 100 * direction + n + oc)
    G = 32 // bs
    mb, kb = 5 * G + 3, 160
    rp, ci, vb = _grouped_small_bsr(rng, bs, mb, kb)
    if direction == 1:
        vb = np.ascontiguousarray(vb.transpose(0, 2, 1))  # the same blocks stored by column
    v = vb.reshape(-1)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    m = mb * bs
    oc_ = ops.ORDER_COL if oc else ops.ORDER_ROW
    ldc = m if oc else n
    for alpha, beta in ((1.0, 0.0), (0.5, -2.0)):
        C0 = rng.uniform(-1, 1, m * n).astype(np.float32)
        dC = _dev(C0)[0] if beta else torch.full((m * n,), float("nan"), device=device)
        ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=ldc, alpha=alpha,
                  beta=beta, direction=direction, order_c=oc_, handle=h)
        torch.cuda.synchronize()
        want = oracle_bsrmm_f32(oracle, direction, mb, n, bs, rp, ci, v, B, n, 0, alpha, beta,
                                C0 if beta else None, ldc, oc)
        got = dC.cpu().numpy()
        assert (got == want).all(), f"bs {bs}: {int((got != want).sum())} elements differ"


@pytest.mark.parametrize("bs", [2, 8])
@pytest.mark.parametrize("n,ldb,ldc,order_b", [(4, 4, 4, 0), (68, 72, 76, 0), (200, 200, 204, 0),
                                               (132, 0, 132, 1)])
def test_small_bs_grouped_shapes(oracle, device, bs, n, ldb, ldc, order_b):
    """The grouped small-bs stream at output widths that are not a whole 128-column
    tile (4, 68, 200, 132), with leading dimensions past n and a column-major B
    (staged row-major first): bit-exact with the sequential oracle."""
    ops = _ops()
    h = _grouped_handle()
    rng = np.random.default_rng(31 * bs + n)
    G = 32 // bs
    mb, kb = 3 * G + 1, 70
    rp, ci, vb = _grouped_small_bsr(rng, bs, mb, kb)
    v = vb.reshape(-1)
    k = kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    if order_b == 0:
        Bd = np.zeros((k, ldb), np.float32)
        Bd[:, :n] = B
        ldbx = ldb
    else:
        Bd = np.ascontiguousarray(B.T)
        ldbx = k
    drp, dci, dv, dB = _dev(rp, ci, v, Bd.reshape(-1))
    m = mb * bs
    dC = torch.full((m * ldc,), float("nan"), device=device)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=ldbx, C=dC, ldc=ldc,
              order_b=ops.ORDER_COL if order_b else ops.ORDER_ROW, handle=h)
    torch.cuda.synchronize()
    want = oracle_bsrmm_f32(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0).reshape(m, n)
    got = dC.cpu().numpy().reshape(m, ldc)[:, :n]
    assert (got == want).all(), f"bs {bs} n {n}: {int((got != want).sum())} elements differ"


@pytest.mark.parametrize("bs", [2, 4, 8])
def test_small_bs_grouped_mixed_sharing(oracle, device, bs):
    """Groups whose block rows share their block columns stay on the grouped
    stream and groups of uniform-random rows (little sharing) are handed to
    bsr_small_kernel: one matrix holding both is bit-exact with the sequential
    oracle, with alpha / beta."""
    ops = _ops()
    h = _grouped_handle()
    rng = np.random.default_rng(900 + bs)
    G = 32 // bs
    mb, kb, n = 8 * G, 400, 128
    rows = []
    for br in range(mb):
        if (br // G) % 2 == 0:   # a band shared by the group
            c = np.unique((br // G) * 13 + rng.integers(0, 40, 30))
        else:                    # uniform random
            c = np.unique(rng.integers(0, kb, 30))
        rows.append(np.sort(c % kb))
    rp = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1] * bs * bs).astype(np.float32)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, mb * bs * n).astype(np.float32)
    drp, dci, dv, dB, dC = _dev(rp, ci, v, B.reshape(-1), C0)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, alpha=0.75,
              beta=0.5, handle=h)
    torch.cuda.synchronize()
    want = oracle_bsrmm_f32(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0, 0.75, 0.5, C0, n, 0)
    got = dC.cpu().numpy()
    assert (got == want).all(), f"bs {bs}: {int((got != want).sum())} elements differ"


@pytest.mark.parametrize("bs", [2, 4, 8])
def test_small_bs_grouped_nonfinite_contract(oracle, device, bs):
    """inf / NaN B rows on the grouped stream: column-granular exactly (an
    element is non-finite iff its block row stores a block whose column meets a
    non-finite B value with a value in it), whatever the other block rows of its
    group hold; every other element bit-identical to the run on B with those
    rows zeroed (the flagged tiles are recomputed by bsr_small_kernel)."""
    ops = _ops()
    h = _grouped_handle()
    rng = np.random.default_rng(77 + bs)
    mb, kb, n = 6 * (32 // bs) + 1, 120, 256
    rp, ci, vb = _grouped_small_bsr(rng, bs, mb, kb)
    v = vb.reshape(-1)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    # rows a stored block uses (a value in its column) and rows only empty columns meet
    used = np.zeros(kb * bs, bool)
    for k in range(rp[-1]):
        used[ci[k] * bs + np.nonzero(np.any(vb[k] != 0, axis=0))[0]] = True
    bad_used = rng.choice(np.nonzero(used)[0], 3, replace=False)
    bad_unused = rng.choice(np.nonzero(~used)[0], 2, replace=False)
    Bbad = B.copy()
    Bbad[bad_used[0], 5] = np.inf
    Bbad[bad_used[1], :] = np.nan
    Bbad[bad_used[2], 130:140] = -np.inf
    Bbad[bad_unused] = np.nan
    Bz = np.where(np.isfinite(Bbad), Bbad, np.float32(0.0))
    want = oracle_bsrmm_f32(oracle, 0, mb, n, bs, rp, ci, v, Bz, n, 0).reshape(mb * bs, n)
    expect_nf = np.zeros((mb * bs, n), bool)
    for br in range(mb):
        for k in range(rp[br], rp[br + 1]):
            for c in np.nonzero(np.any(vb[k] != 0, axis=0))[0]:
                expect_nf[br * bs:(br + 1) * bs] |= ~np.isfinite(Bbad[ci[k] * bs + c])[None, :]
    assert expect_nf.any()
    drp, dci, dv, dB = _dev(rp, ci, v, Bbad.reshape(-1))
    dC = torch.full((mb * bs * n,), 7.0, device=device)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, handle=h)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape(mb * bs, n)
    assert np.array_equal(~np.isfinite(got), expect_nf), "non-finite pattern"
    assert (got[~expect_nf] == want[~expect_nf]).all(), "finite elements"


@pytest.mark.parametrize("bs", [2, 8])
def test_small_bs_grouped_unsorted_columns(oracle, device, bs):
    """Block columns out of order inside rows (and so not sharing batches):
    the grouped stream still multiplies every block, within the fp32 bar of the
    f64 oracle."""
    ops = _ops()
    h = _grouped_handle()
    rng = np.random.default_rng(55 + bs)
    mb, kb, n = 4 * (32 // bs) + 2, 90, 128
    rp, ci, vb = _grouped_small_bsr(rng, bs, mb, kb, sorted_cols=False)
    v = vb.reshape(-1)
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B.reshape(-1))
    dC = torch.full((mb * bs * n,), float("nan"), device=device)
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=dC, ldc=n, handle=h)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    assert_normwise(dC.cpu().numpy().reshape(mb * bs, n), ref, absd, TOL_F32, f"bs {bs} unsorted")


@pytest.mark.parametrize("n,oc", [(128, 0), (256, 0), (96, 1)])
def test_bsr64_matches_bs32_sub_blocks(oracle, device, n, oc):
    """bs 64 runs the bs 32 column stream on each block's 32 x 32 sub-blocks:
    C is bit-identical to the bs 32 kernel on the same matrix cut at bs 32
    (device csr2bsr of the same CSR: its sub-blocks, in block-column order,
    the all-zero ones dropped, which the stream skips anyway), and within the
    bar of the f64 oracle."""
    ops = _ops()
    rng = np.random.default_rng(640 + n + oc)
    m = 64 * 41
    # dense-ish diagonal regions plus one scattered entry per row: fewer than 64
    # blocks per bs 32 block row, so the bs 32 launch cuts no row into segments
    rows = []
    for r in range(m):
        dense = (r // 32) * 32 + rng.choice(32, 12, replace=False)
        rows.append(np.unique(np.concatenate([dense, rng.choice(m, 1)])))
    rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    B = torch.rand((m, n), device=device) * 2 - 1
    outs = []
    for bs in (64, 32):
        brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=m, n=m, bs=bs)
        mb = m // bs
        C = torch.full((m, n), float("nan"), device=device) if oc == 0 else \
            torch.full((n, m), float("nan"), device=device)
        ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=n, bs=bs, ldb=n, C=C, ldc=n if oc == 0 else m,
                  order_c=oc)
        torch.cuda.synchronize()
        outs.append(C if oc == 0 else C.t())
    assert torch.equal(outs[0], outs[1]), "bs 64 differs from the bs 32 sub-block stream"
    ref, absd = oracle_csrmm_f64(oracle, m, n, rp, ci, v, B.cpu().numpy(), n, 0)
    assert_normwise(outs[0].cpu().numpy(), ref, absd, TOL_F32, f"bs 64 n={n}")


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("n,ob,oc,alpha,beta", [(256, 0, 0, 1.0, 0.0), (512, 0, 0, 0.5, -1.0),
                                                (136, 0, 1, 1.0, 0.0), (264, 1, 0, 2.0, 0.5)])
def test_bsrmm_grouped_f16(oracle, device, W, n, ob, oc, alpha, beta):
    """The grouped bs 16 fp16 stream (spmm_bsr16_group_analysis_f16 +
    spmm_bsrmm_grouped_f16): groups of W block rows sharing the union of their
    columns, an mb that W does not divide, empty block rows and blocks, empty
    columns; against the f64 oracle of the same fp16 values, alpha / beta,
    column-major B (staged) and C."""
    ops = _ops()
    rng = np.random.default_rng(16 * W + n + ob)
    mb, kb = 37, 60
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, 16, 0.3)
    v16 = v.astype(np.float16)
    Bd = rng.uniform(-1, 1, (kb * 16, n)).astype(np.float16)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    m = mb * 16
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    Ch = C0 if oc == 0 else np.ascontiguousarray(C0.T)
    drp, dci, dv, dB, dC = _dev(rp, ci, v16, B.reshape(-1), Ch.reshape(-1))
    grp = ops.GroupedBsr16(drp, dci, dv, mb=mb, group_rows=W)
    grp.mm(dB, kb=kb, n=n, ldb=n if ob == 0 else kb * 16, order_b=ob, C=dC,
           ldc=n if oc == 0 else m, order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape((m, n) if oc == 0 else (n, m))
    got = got if oc == 0 else got.T
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, 16, rp, ci, v16, Bd, n, 0, half=True)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(got, ref, absd, TOL_F16_ACC, f"grouped W={W} n={n} ob={ob} oc={oc}")
    grp.close()


def colgran_nonfinite_block_rows(rp, ci, v, bs, mb, bad_rows):
    """The column-granular non-finite contract (include/spmm_hip.h), predicted
    from the pattern on the host: a non-finite B row J * bs + c reaches every
    row of block row I iff I stores block column J with a value other than +-0
    in its column c; no other row. v: [nnzb, bs, bs] row-major block values.
    Returns a bool per block row."""
    held = np.zeros(mb, bool)
    blk_row = np.repeat(np.arange(mb), np.diff(rp))
    for b in bad_rows:
        J, c = divmod(int(b), bs)
        k = np.nonzero(ci == J)[0]
        k = k[(v[k, :, c] != 0).any(axis=1)]
        held[blk_row[k]] = True
    return held


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("bad", ["nan", "inf"])
def test_bsrmm_grouped_f16_nonfinite_contract(device, W, bad):
    """An inf / NaN in B through the grouped stream: the contract is the drop-in
    stream's column-granular one (round 5; round 4's GROUPED contract spread it
    to the whole group). Exactly the block rows colgran_nonfinite_block_rows
    predicts are non-finite in every element; another block row of the same
    group stays finite and equals the run on B with those rows zeroed, bit for
    bit; a column whose blocks hold it only as zeros and a column no block
    stores reach no row. The case must have groups that contain both a hit and
    a spared block row (where the two contracts differ)."""
    ops = _ops()
    rng = np.random.default_rng(7 * W + (bad == "inf"))
    mb, kb, n = 37, 60, 256
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, 16, 0.3)
    v16 = v.astype(np.float16)
    B = rng.uniform(-1, 1, (kb * 16, n)).astype(np.float16)
    vb = v16.astype(np.float32).reshape(-1, 16, 16)
    col_nz = np.zeros((kb, 16), bool)
    col_st = np.zeros(kb, bool)
    col_st[ci] = True
    for k, J in enumerate(ci):
        col_nz[J] |= (vb[k] != 0).any(axis=0)
    held = np.argwhere(col_nz)
    zero_only = np.argwhere(~col_nz & col_st[:, None])
    unstored = np.nonzero(~col_st)[0]
    bad_rows = [int(held[len(held) // 2][0]) * 16 + int(held[len(held) // 2][1])]
    if len(zero_only):
        bad_rows.append(int(zero_only[0][0]) * 16 + int(zero_only[0][1]))
    if len(unstored):
        bad_rows.append(int(unstored[0]) * 16 + 5)
    want = colgran_nonfinite_block_rows(rp, ci, vb, 16, mb, bad_rows)
    grp_any = np.pad(want, (0, -mb % W)).reshape(-1, W).any(axis=1)
    assert 0 < want.sum() < np.repeat(grp_any, W)[:mb].sum(), (
        "the case must have a group with both a hit and a spared block row")
    B0 = B.copy()
    B0[bad_rows] = 0
    B[bad_rows] = np.float16(np.nan if bad == "nan" else np.inf)
    drp, dci, dv = _dev(rp, ci, v16)
    grp = ops.GroupedBsr16(drp, dci, dv, mb=mb, group_rows=W)
    outs = []
    for Bx in (B, B0):
        C = torch.zeros((mb * 16, n), device=device)
        grp.mm(torch.from_numpy(Bx).to(device), kb=kb, n=n, ldb=n, C=C, ldc=n)
        outs.append(C)
    torch.cuda.synchronize()
    grp.close()
    bad_el = ~torch.isfinite(outs[0]).view(mb, 16 * n)
    w = torch.from_numpy(want).to(device)
    assert torch.equal(bad_el.any(dim=1), w) and torch.equal(bad_el.all(dim=1), w), (
        f"W={W} {bad}: non-finite block rows {int(bad_el.any(dim=1).sum())} "
        f"(whole: {int(bad_el.all(dim=1).sum())}), expected {int(want.sum())}")
    keep = ~w.repeat_interleave(16)
    assert torch.equal(outs[0][keep], outs[1][keep]), "finite rows differ from the zeroed-B run"


def test_bsrmm_grouped_f16_checks(device):
    """A buffer this handle holds no analysis of, another mb, or a kb below
    an analysed block column is INVALID_VALUE, and so is a negative block
    column at analysis; n % 8 != 0 is NOT_SUPPORTED (before any launch)."""
    from spmm_hip._lib import INVALID_VALUE, NOT_SUPPORTED, SpmmError
    ops = _ops()
    rng = np.random.default_rng(3)
    rp, ci, v = _column_sparse_bsr(rng, 5, 7, 16, 0.5)
    drp, dci, dv = _dev(rp, ci, v.astype(np.float16))
    grp = ops.GroupedBsr16(drp, dci, dv, mb=5)
    B = torch.zeros((7 * 16, 128), dtype=torch.float16, device=device)
    C = torch.zeros((5 * 16, 128), device=device)
    grp.mb = 6
    with pytest.raises(SpmmError) as e:
        grp.mm(B, kb=7, n=128, ldb=128, C=C, ldc=128)
    assert e.value.status == INVALID_VALUE
    grp.mb = 5
    with pytest.raises(SpmmError) as e:
        grp.mm(B, kb=7, n=124, ldb=128, C=C, ldc=128)
    assert e.value.status == NOT_SUPPORTED
    # a kb the analysed block columns do not fit would read B past its rows
    with pytest.raises(SpmmError) as e:
        grp.mm(B, kb=int(ci.max()), n=128, ldb=128, C=C, ldc=128)
    assert e.value.status == INVALID_VALUE
    grp.close()
    bad = ci.copy()
    bad[0] = -1
    with pytest.raises(SpmmError) as e:  # a negative block column
        ops.GroupedBsr16(drp, torch.from_numpy(bad).to(device), dv, mb=5)
    assert e.value.status == INVALID_VALUE
    with pytest.raises(SpmmError) as e:  # released: the handle no longer knows the buffer
        grp.buffer = torch.empty(16, dtype=torch.uint8, device=device)
        grp.mm(B, kb=7, n=128, ldb=128, C=C, ldc=128)
    assert e.value.status == INVALID_VALUE


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("n,ob,oc,alpha,beta,direction",
                         [(128, 0, 0, 1.0, 0.0, 0), (256, 0, 0, 0.5, -1.0, 0), (64, 0, 0, 1.0, 0.0, 1),
                          (132, 0, 1, 1.0, 0.0, 0), (260, 1, 0, 2.0, 0.5, 1), (128, 1, 1, 1.0, 1.0, 0)])
def test_bsrmm_grouped_f32(oracle, device, W, n, ob, oc, alpha, beta, direction):
    """The grouped bs 32 fp32 stream (spmm_bsr32_group_analysis_f32 +
    spmm_bsrmm_grouped_f32): groups of W block rows sharing the union of their
    columns, each multiplying only its own nonzero columns. An mb that W does not
    divide, empty block rows, explicit zero blocks, single-column blocks, ROW and
    COLUMN blocks, partial column tiles, alpha / beta, column-major B and C (staged);
    against the f64 oracle, and bit-identical to spmm_bsrmm_ex_f32 (the same MFMAs
    in the same order) where both run row-major."""
    from spmm_hip._lib import DIRECTION_COLUMN, DIRECTION_ROW
    ops = _ops()
    rng = np.random.default_rng(32 * W + n + 7 * ob + direction)
    mb, kb = 37, 60
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, 32, 0.3)
    vd = v if direction == 0 else np.ascontiguousarray(v.reshape(-1, 32, 32).transpose(0, 2, 1)).reshape(-1)
    dr = DIRECTION_ROW if direction == 0 else DIRECTION_COLUMN
    Bd = rng.uniform(-1, 1, (kb * 32, n)).astype(np.float32)
    B = Bd if ob == 0 else np.ascontiguousarray(Bd.T)
    m = mb * 32
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    Ch = C0 if oc == 0 else np.ascontiguousarray(C0.T)
    drp, dci, dv, dB, dC = _dev(rp, ci, vd, B.reshape(-1), Ch.reshape(-1))
    grp = ops.GroupedBsr32(drp, dci, dv, mb=mb, group_rows=W, direction=dr)
    grp.mm(dB, kb=kb, n=n, ldb=n if ob == 0 else kb * 32, order_b=ob, C=dC,
           ldc=n if oc == 0 else m, order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got = dC.cpu().numpy().reshape((m, n) if oc == 0 else (n, m))
    got = got if oc == 0 else got.T
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, 32, rp, ci, v, Bd, n, 0)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(got, ref, absd, TOL_F32, f"grouped bs32 W={W} n={n} ob={ob} oc={oc}")
    if ob == 0 and oc == 0 and n % 128 == 0:
        Cd = torch.from_numpy(C0.copy()).to(device)
        ops.bsrmm(drp, dci, dv, torch.from_numpy(Bd).to(device), mb=mb, kb=kb, n=n, bs=32, ldb=n,
                  C=Cd, ldc=n, alpha=alpha, beta=beta, direction=dr)
        torch.cuda.synchronize()
        assert torch.equal(Cd.cpu(), torch.from_numpy(got)), "grouped bs 32 differs from bsrmm"
    grp.close()


@pytest.mark.parametrize("bs", [32, 16])
def test_group_analysis_size_query_recomputes(device, bs):
    """A size query abandoned on one matrix, then the values changed in place
    (same addresses, other zero columns, as a caching allocator hands out), a
    new size query and the fill: the buffer equals a fresh handle's analysis of
    the new values byte for byte (every size query recomputes; group.cpp)."""
    from ctypes import byref, c_size_t
    from spmm_hip._lib import lib
    ops = _ops()
    rng = np.random.default_rng(77 + bs)
    mb, kb = 23, 30
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.3)
    nnzb = ci.size
    keep = rng.random((nnzb, 1, bs)) >= 0.6  # other columns of every block zero
    v2 = (rng.uniform(-1, 1, (nnzb, bs, bs)) * keep).astype(np.float32).reshape(-1)
    vt = np.float16 if bs == 16 else np.float32
    drp, dci, dv = _dev(rp, ci, v.astype(vt))
    h, fresh_h = ops.Handle(), ops.Handle()
    fn = getattr(lib(), "spmm_bsr16_group_analysis_f16" if bs == 16 else
                 "spmm_bsr32_group_analysis_f32")
    grp_cls = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32

    def args():
        return (h.raw, ops.DIRECTION_ROW, mb, nnzb, 2, ops._ptr(drp), ops._ptr(dci), ops._ptr(dv))
    size = c_size_t(0)
    assert fn(*args(), None, byref(size)) == 0  # the query on the first values, abandoned
    dv.copy_(torch.from_numpy(v2.astype(vt)))
    size2 = c_size_t(0)
    assert fn(*args(), None, byref(size2)) == 0
    buf = torch.empty(max(size2.value, 1), dtype=torch.uint8, device=device)
    assert fn(*args(), ops._ptr(buf), byref(size2)) == 0
    fresh = grp_cls(drp, dci, dv, mb=mb, group_rows=2, handle=fresh_h)
    torch.cuda.synchronize()
    assert size2.value == fresh.bytes
    assert torch.equal(buf[:size2.value], fresh.buffer[:fresh.bytes])
    lib().spmm_bsr_group_release(h.raw, ops._ptr(buf))
    fresh.close()
    h.close()
    fresh_h.close()


def test_bsrmm_grouped_f32_checks(device):
    """A bs 16 analysis is not a bs 32 one; another mb, a kb below an analysed
    block column, a buffer without an analysis are INVALID_VALUE; W = 8 is
    INVALID_VALUE at bs 32; n % 4 != 0 is NOT_SUPPORTED."""
    from spmm_hip._lib import INVALID_VALUE, NOT_SUPPORTED, SpmmError
    ops = _ops()
    rng = np.random.default_rng(5)
    rp, ci, v = _column_sparse_bsr(rng, 5, 7, 32, 0.5)
    drp, dci, dv = _dev(rp, ci, v)
    grp = ops.GroupedBsr32(drp, dci, dv, mb=5)
    B = torch.zeros((7 * 32, 128), device=device)
    C = torch.zeros((5 * 32, 128), device=device)
    grp.mm(B, kb=7, n=128, ldb=128, C=C, ldc=128)
    for kw, status in ((dict(kb=7, n=126, ldb=128), NOT_SUPPORTED),
                       (dict(kb=int(ci.max()), n=128, ldb=128), INVALID_VALUE)):
        with pytest.raises(SpmmError) as e:
            grp.mm(B, C=C, ldc=128, **kw)
        assert e.value.status == status, kw
    grp.mb = 6
    with pytest.raises(SpmmError) as e:
        grp.mm(B, kb=7, n=128, ldb=128, C=C, ldc=128)
    assert e.value.status == INVALID_VALUE
    grp.mb = 5
    grp.close()
    with pytest.raises(SpmmError) as e:
        ops.GroupedBsr32(drp, dci, dv, mb=5, group_rows=8)
    assert e.value.status == INVALID_VALUE
    # a bs 16 analysis buffer is refused by the bs 32 product
    rp16, ci16, v16 = _column_sparse_bsr(rng, 5, 7, 16, 0.5)
    d16 = _dev(rp16, ci16, v16.astype(np.float16))
    g16 = ops.GroupedBsr16(*d16, mb=5)
    grp.buffer = g16.buffer
    with pytest.raises(SpmmError) as e:
        grp.mm(B, kb=7, n=128, ldb=128, C=C, ldc=128)
    assert e.value.status == INVALID_VALUE
    g16.close()


def test_grouped_streams_random_shapes(oracle, device):
    """Both grouped streams over random small shapes: mb from 1 (a single, partial
    group) to 45, every W, block rows with no blocks, n at and around the tile
    widths, beta != 0; against the f64 oracle (bs 32 also bit-identical to
    spmm_bsrmm_ex_f32 where both run row-major)."""
    ops = _ops()
    rng = np.random.default_rng(2024)
    for case in range(16):
        bs = 16 if case % 2 == 0 else 32
        W = int(rng.choice([2, 4, 8] if bs == 16 else [2, 4]))
        mb = int(rng.integers(1, 46))
        kb = int(rng.integers(1, 50))
        n = int(rng.choice([8, 16, 120, 256, 264]) if bs == 16 else rng.choice([4, 64, 128, 132, 256]))
        rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, float(rng.uniform(0.05, 0.6)))
        half = bs == 16
        vv = v.astype(np.float16) if half else v
        Bd = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float16 if half else np.float32)
        C0 = rng.uniform(-1, 1, (mb * bs, n)).astype(np.float32)
        drp, dci, dv, dB, dC = _dev(rp, ci, vv, Bd.reshape(-1), C0.reshape(-1))
        G = ops.GroupedBsr16 if half else ops.GroupedBsr32
        grp = G(drp, dci, dv, mb=mb, group_rows=W)
        grp.mm(dB, kb=kb, n=n, ldb=n, C=dC, ldc=n, alpha=1.5, beta=0.5)
        torch.cuda.synchronize()
        got = dC.cpu().numpy().reshape(mb * bs, n)
        ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, vv, Bd, n, 0, half=half)
        ref = 1.5 * ref + 0.5 * C0.astype(np.float64)
        absd = 1.5 * absd + 0.5 * np.abs(C0.astype(np.float64))
        what = f"case {case}: bs {bs} W {W} mb {mb} kb {kb} n {n}"
        assert_normwise(got, ref, absd, TOL_F16_ACC if half else TOL_F32, what)
        if not half:
            Cd = torch.from_numpy(C0.copy()).to(device)
            ops.bsrmm(drp, dci, dv, torch.from_numpy(Bd).to(device), mb=mb, kb=kb, n=n, bs=32,
                      ldb=n, C=Cd, ldc=n, alpha=1.5, beta=0.5)
            torch.cuda.synchronize()
            assert torch.equal(Cd.cpu(), torch.from_numpy(got)), what + ": differs from bsrmm"
        grp.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_grouped_streams_empty_matrix(device, bs):
    """A matrix with block rows but no blocks: the analysis makes no items and the product
    leaves C = beta C (the padding of every group empty); mb = 0 is a quick success."""
    ops = _ops()
    mb, kb, n = 7, 5, 128
    rp = np.zeros(mb + 1, np.int32)
    ci = np.zeros(0, np.int32)
    v = np.zeros(0, np.float16 if bs == 16 else np.float32)
    drp, dci = torch.from_numpy(rp).to(device), torch.from_numpy(ci).to(device)
    dv = torch.from_numpy(v).to(device)
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    grp = G(drp, dci, dv, mb=mb)
    B = torch.ones((kb * bs, n), dtype=torch.float16 if bs == 16 else torch.float32, device=device)
    C = torch.full((mb * bs, n), 2.0, device=device)
    grp.mm(B, kb=kb, n=n, ldb=n, C=C, ldc=n, alpha=1.0, beta=0.5)
    torch.cuda.synchronize()
    assert torch.equal(C, torch.full_like(C, 1.0))
    grp.close()
    g0 = G(torch.zeros(1, dtype=torch.int32, device=device), dci, dv, mb=0)
    g0.mm(B, kb=kb, n=n, ldb=n, C=C, ldc=n)
    g0.close()


@pytest.mark.parametrize("bs,W", [(16, 2), (16, 4), (16, 8), (32, 2), (32, 4)])
def test_group_analysis_layout(device, bs, W):
    """The device group analysis against a numpy restatement of the grouping: per group of
    W block rows, the union of their blocks' nonzero columns in (block column, column)
    order, cut into items of 16 (bs 16) or 8 (bs 32) entries, the last padded with -1. The
    buffer's item pointers and entry rows must be exactly that (include/spmm_hip.h layout:
    256-B header, item_ptr[ngroups + 1], rows[nitems][E] at the next 256-B boundary)."""
    ops = _ops()
    rng = np.random.default_rng(100 * bs + W)
    mb, kb = 29, 40
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.35)
    E = 16 if bs == 16 else 8
    vv = v.astype(np.float16) if bs == 16 else v
    vb = vv.astype(np.float32).reshape(-1, bs, bs)  # ROW blocks: [block][row][column]
    nz_cols = [np.nonzero((np.abs(vb[k]) > 0).any(axis=0))[0] for k in range(vb.shape[0])]
    ngroups = (mb + W - 1) // W
    want_ptr, want_rows = [0], []
    for g in range(ngroups):
        ent = set()
        for br in range(g * W, min(mb, g * W + W)):
            for k in range(rp[br], rp[br + 1]):
                ent.update(int(ci[k]) * bs + int(c) for c in nz_cols[k])
        ent = sorted(ent)
        ent += [-1] * (-len(ent) % E)
        want_rows += ent
        want_ptr.append(want_ptr[-1] + len(ent) // E)
    drp, dci, dv = _dev(rp, ci, vv)
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    grp = G(drp, dci, dv, mb=mb, group_rows=W)
    buf = grp.buffer.cpu().numpy()
    ptr = buf[256:256 + 4 * (ngroups + 1)].view(np.int32)
    assert np.array_equal(ptr, np.array(want_ptr, np.int32)), "item pointers"
    rows_off = (256 + 4 * (ngroups + 1) + 255) // 256 * 256
    got_rows = buf[rows_off:rows_off + 4 * len(want_rows)].view(np.int32)
    assert np.array_equal(got_rows, np.array(want_rows, np.int32)), "entry rows"
    grp.close()


def _long_row_bsr(rng, mb, kb, bs, lengths):
    """Block rows of the given lengths (block columns drawn sorted from kb) whose
    blocks hold a random set of nonzero columns (about 30 %, none in some blocks)."""
    counts = rng.choice(lengths, mb)
    rp = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(kb, c, replace=False)) for c in counts] +
                        [np.zeros(0, np.int64)]).astype(np.int32)
    nnzb = int(rp[-1])
    active = rng.random((nnzb, bs)) < 0.3
    active[::7] = False  # explicit all-zero blocks
    v = rng.uniform(-1, 1, (nnzb, bs, bs)) * (rng.random((nnzb, bs, bs)) < 0.3)
    v[np.arange(nnzb)[:, None], rng.integers(bs, size=(nnzb, bs)), np.arange(bs)[None, :]] = 0.5
    v = (v * active[:, None, :]).astype(np.float32)  # ROW blocks: [block][row][column]
    return rp, ci, v.reshape(-1), active


@pytest.mark.parametrize("bs,W", [(16, 2), (16, 4), (16, 8), (32, 2), (32, 4)])
def test_group_analysis_layout_long_rows(device, bs, W):
    """The device merge (group_kernels.hip, one wave per group, windows of 64 / W block
    columns per row) on rows far longer than a window and of very different lengths in
    one group (0 .. 600 blocks): item pointers, entry rows and the per-(item, wave) held
    masks equal the numpy restatement of the grouping."""
    ops = _ops()
    rng = np.random.default_rng(7 * bs + W)
    mb, kb = 37, 600
    rp, ci, v, active = _long_row_bsr(rng, mb, kb, bs, [0, 1, 3, 17, 40, 200, 600])
    E = 16 if bs == 16 else 8
    vv = v.astype(np.float16) if bs == 16 else v
    ngroups = (mb + W - 1) // W
    want_ptr, want_rows, want_wm = [0], [], []
    for g in range(ngroups):
        held = []
        for br in range(g * W, g * W + W):
            h = set()
            if br < mb:
                for k in range(rp[br], rp[br + 1]):
                    h.update(int(ci[k]) * bs + int(c) for c in np.nonzero(active[k])[0])
            held.append(h)
        ent = sorted(set().union(*held))
        ent += [-1] * (-len(ent) % E)
        for it in range(len(ent) // E):
            for w in range(W):
                want_wm.append(sum(1 << e for e in range(E) if ent[it * E + e] in held[w]))
        want_rows += ent
        want_ptr.append(want_ptr[-1] + len(ent) // E)
    drp, dci, dv = _dev(rp, ci, vv)
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    grp = G(drp, dci, dv, mb=mb, group_rows=W)
    buf = grp.buffer.cpu().numpy()
    ptr = buf[256:256 + 4 * (ngroups + 1)].view(np.int32)
    assert np.array_equal(ptr, np.array(want_ptr, np.int32)), "item pointers"
    rows_off = (256 + 4 * (ngroups + 1) + 255) // 256 * 256
    got_rows = buf[rows_off:rows_off + 4 * len(want_rows)].view(np.int32)
    assert np.array_equal(got_rows, np.array(want_rows, np.int32)), "entry rows"
    wm_off = (rows_off + 4 * len(want_rows) + 255) // 256 * 256
    got_wm = buf[wm_off:wm_off + 4 * len(want_wm)].view(np.uint32)
    assert np.array_equal(got_wm, np.array(want_wm, np.uint32)), "held-entry masks"
    # the A fragments (fill kernels): A[r][c] of the block of row w holding (J, c), zero
    # where that row holds no such nonzero column or the entry is padding
    nitems = len(want_rows) // E
    af_off = (wm_off + 4 * nitems * W + 255) // 256 * 256
    ent = np.array(want_rows, np.int64).reshape(nitems, E)
    item_group = np.repeat(np.arange(ngroups), np.diff(want_ptr))
    vb = vv.reshape(-1, bs, bs)
    where = {(br, int(ci[k])): k for br in range(mb) for k in range(rp[br], rp[br + 1])}
    want_af = np.zeros((nitems, W, bs, E), vb.dtype)  # [item][w][row][entry]
    for w in range(W):
        held = np.array(want_wm, np.int64).reshape(nitems, W)[:, w]
        for it, e in zip(*np.nonzero((held[:, None] >> np.arange(E)) & 1)):
            J, c = divmod(int(ent[it, e]), bs)
            want_af[it, w, :, e] = vb[where[(int(item_group[it]) * W + w, J)], :, c]
    if bs == 32:
        got_af = buf[af_off:af_off + 4 * want_af.size].view(np.float32).reshape(want_af.shape)
    else:  # half 64 (e >> 2) + 4 r + (e & 3) of each (item, w)
        raw = buf[af_off:af_off + 2 * want_af.size].view(np.float16).reshape(nitems, W, 256)
        r_, e_ = np.meshgrid(np.arange(16), np.arange(16), indexing="ij")
        got_af = raw[:, :, 64 * (e_ >> 2) + 4 * r_ + (e_ & 3)]
    assert np.array_equal(got_af.view(np.uint32 if bs == 32 else np.uint16),
                          want_af.view(np.uint32 if bs == 32 else np.uint16)), "A fragments"
    grp.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_group_analysis_column_blocks(device, bs):
    """A matrix given as COLUMN blocks (each block stored transposed) gives the same
    analysis buffer, byte for byte, as the same matrix given as ROW blocks: the fill
    kernels read either layout."""
    from spmm_hip._lib import DIRECTION_COLUMN
    ops = _ops()
    rng = np.random.default_rng(55 + bs)
    mb, kb = 21, 300
    rp, ci, v, _ = _long_row_bsr(rng, mb, kb, bs, [0, 2, 9, 60, 150])
    vv = v.astype(np.float16) if bs == 16 else v
    vcol = np.ascontiguousarray(vv.reshape(-1, bs, bs).transpose(0, 2, 1)).reshape(-1)
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    W = 4 if bs == 16 else 2
    drp, dci, dv = _dev(rp, ci, vv)
    a = G(drp, dci, dv, mb=mb, group_rows=W)
    want = a.buffer.cpu().numpy().copy()
    a.close()
    drp, dci, dvc = _dev(rp, ci, vcol)
    b = G(drp, dci, dvc, mb=mb, group_rows=W, direction=DIRECTION_COLUMN)
    assert np.array_equal(b.buffer.cpu().numpy(), want)
    b.close()


@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("fault", ["duplicate", "descending", "negative"])
def test_group_analysis_rejects_unsorted_block_columns(device, bs, fault):
    """Block columns must be strictly increasing within a block row (include/spmm_hip.h):
    a duplicate, a descending pair (within a merge window and across windows) or a
    negative block column is INVALID_VALUE from the size query, with no fault; the same
    handle then analyses the good matrix."""
    from spmm_hip._lib import INVALID_VALUE, SpmmError
    ops = _ops()
    rng = np.random.default_rng(31 + bs)
    mb, kb = 9, 300
    rp, ci, v, _ = _long_row_bsr(rng, mb, kb, bs, [120])
    vv = v.astype(np.float16) if bs == 16 else v
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    h = ops.Handle()
    for at in (5, 32, 100):  # inside the first window, at a window edge, past it
        b = ci.copy()
        k = int(rp[4]) + at
        if fault == "duplicate":
            b[k] = b[k - 1]
        elif fault == "descending":
            b[k - 1], b[k] = b[k], b[k - 1]
        else:
            b[k] = -3
        drp, dci, dv = _dev(rp, b, vv)
        with pytest.raises(SpmmError) as e:
            G(drp, dci, dv, mb=mb, handle=h)
        assert e.value.status == INVALID_VALUE
    drp, dci, dv = _dev(rp, ci, vv)
    G(drp, dci, dv, mb=mb, handle=h).close()
    torch.cuda.synchronize()
    h.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_group_analysis_row_pointer_checked_on_device(device, bs):
    """The group analysis checks the row pointer on the device (grp_build_kernel
    PASS 1) before it indexes the block columns: rp[0] != 0, a decreasing entry,
    an entry past nnzb and rp[mb] != nnzb are each INVALID_VALUE from the size
    query, with no fault; the same handle then analyses a good matrix."""
    from spmm_hip._lib import INVALID_VALUE, SpmmError
    ops = _ops()
    rng = np.random.default_rng(9 + bs)
    mb, kb = 23, 30
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.3)
    vv = v.astype(np.float16) if bs == 16 else v
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    nnzb = int(rp[-1])
    bads = []
    for fix in ("first", "decrease", "past", "last"):
        b = rp.copy()
        if fix == "first":
            b[0] = 1
        elif fix == "decrease":
            b[mb // 2] = b[mb // 2 + 1] + 1
        elif fix == "past":
            b[mb // 2] = nnzb + 1000
        else:
            b[mb] = nnzb - 1
        bads.append(b)
    h = ops.Handle()
    for b in bads:
        drp, dci, dv = _dev(b, ci, vv)
        with pytest.raises(SpmmError) as e:
            G(drp, dci, dv, mb=mb, handle=h)
        assert e.value.status == INVALID_VALUE
    drp, dci, dv = _dev(rp, ci, vv)
    G(drp, dci, dv, mb=mb, handle=h).close()
    torch.cuda.synchronize()
    h.close()


@pytest.mark.parametrize("W", [2, 4])
def test_group32_one_pass_fill_equals_block_fill(device, W):
    """The bs 32 analysis in one pass over A (group_kernels.hip: the masks' kernel leaves a
    compact copy of ROW blocks' nonzero columns, the fill reads 128 B per entry from it)
    writes the same buffer, byte for byte, as the block fill, which reads every held
    block's 4 KB again (run here by capturing the filling call: a captured fill reads the
    values themselves). Some 60 k blocks, rows of 0 .. 400 blocks."""
    from ctypes import byref, c_size_t, c_void_p
    from spmm_hip._lib import lib
    ops = _ops()
    rng = np.random.default_rng(900 + W)
    mb, kb = 1500, 2000
    rp, ci, v, _ = _long_row_bsr(rng, mb, kb, 32, [0, 3, 20, 45, 90, 400])
    drp, dci, dv = _dev(rp, ci, v)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        h = ops.Handle(s)
        ref = ops.GroupedBsr32(drp, dci, dv, mb=mb, group_rows=W, handle=h)  # one pass
        fn = lib().spmm_bsr32_group_analysis_f32
        args = (h.raw, 0, mb, int(ci.size), W, c_void_p(drp.data_ptr()), c_void_p(dci.data_ptr()),
                c_void_p(dv.data_ptr()))
        size = c_size_t(0)
        assert fn(*args, None, byref(size)) == 0 and size.value == ref.bytes
        buf = torch.full((size.value,), 0xA5, dtype=torch.uint8, device=device)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            h.set_stream(s)
            assert fn(*args, c_void_p(buf.data_ptr()), byref(size)) == 0
        g.replay()
        s.synchronize()
        assert torch.equal(buf, ref.buffer[:size.value]), "one-pass fill differs from the block fill"
        ref.close()
        h.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_group_analysis_fill_is_graph_capturable(device, bs):
    """The filling call of the group analysis only launches kernels and async
    copies: after an eager analysis has grown the handle's buffers, a size query
    (eager) followed by the filling call CAPTURED in a HIP graph and replayed
    writes the same buffer, byte for byte, as the eager analysis, and the
    grouped product on it equals the eager one. A filling call after a size
    query of other arguments (another matrix) still analyses its own matrix."""
    from ctypes import byref, c_size_t, c_void_p
    from spmm_hip._lib import lib
    ops = _ops()
    rng = np.random.default_rng(77 + bs)
    mb, kb, n = 41, 50, 128
    rp, ci, v = _column_sparse_bsr(rng, mb, kb, bs, 0.3)
    vv = v.astype(np.float16) if bs == 16 else v
    drp, dci, dv = _dev(rp, ci, vv)
    G = ops.GroupedBsr16 if bs == 16 else ops.GroupedBsr32
    fn = lib().spmm_bsr16_group_analysis_f16 if bs == 16 else lib().spmm_bsr32_group_analysis_f32
    W = 4 if bs == 16 else 2
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        h = ops.Handle(s)
        ref = G(drp, dci, dv, mb=mb, group_rows=W, handle=h)  # eager: grows the buffers
        size = c_size_t(0)
        args = (h.raw, 0, mb, int(ci.size), W, c_void_p(drp.data_ptr()), c_void_p(dci.data_ptr()),
                c_void_p(dv.data_ptr()))
        assert fn(*args, None, byref(size)) == 0 and size.value == ref.bytes
        buf = torch.zeros(size.value, dtype=torch.uint8, device=device)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            h.set_stream(s)
            st = fn(*args, c_void_p(buf.data_ptr()), byref(size))
        assert st == 0
        g.replay()
        s.synchronize()
        assert torch.equal(buf, ref.buffer[:size.value]), "captured fill differs from the eager one"
        # the product on the captured buffer (recorded on the handle at capture)
        vt = torch.float16 if bs == 16 else torch.float32
        B = (torch.rand((kb * bs, n), device=device) * 2 - 1).to(vt)
        C1 = torch.zeros((mb * bs, n), device=device)
        C2 = torch.zeros((mb * bs, n), device=device)
        ref.mm(B, kb=kb, n=n, ldb=n, C=C1, ldc=n)
        pfn = lib().spmm_bsrmm_grouped_f16 if bs == 16 else lib().spmm_bsrmm_grouped_f32
        assert pfn(h.raw, mb, kb, n, c_void_p(buf.data_ptr()), 1.0, c_void_p(B.data_ptr()), n, 0,
                   0.0, c_void_p(C2.data_ptr()), n, 0) == 0
        s.synchronize()
        assert torch.equal(C1, C2)
        # a size query of another matrix, then the filling call of this one
        rp2, ci2, v2 = _column_sparse_bsr(rng, 9, 12, bs, 0.5)
        v2 = v2.astype(np.float16) if bs == 16 else v2
        e_rp, e_ci, e_v = _dev(rp2, ci2, v2)
        other = (h.raw, 0, 9, int(ci2.size), W, c_void_p(e_rp.data_ptr()),
                 c_void_p(e_ci.data_ptr()), c_void_p(e_v.data_ptr()))
        assert fn(*other, None, byref(c_size_t(0))) == 0
        buf2 = torch.zeros(ref.bytes, dtype=torch.uint8, device=device)
        size = c_size_t(ref.bytes)
        assert fn(*args, c_void_p(buf2.data_ptr()), byref(size)) == 0
        s.synchronize()
        assert torch.equal(buf2, ref.buffer[:ref.bytes])
    ref.close()
    for b in (buf, buf2):
        lib().spmm_bsr_group_release(h.raw, c_void_p(b.data_ptr()))
    h.close()


def _reblock32_numpy(rp, ci, v, bs, mb, direction):
    """Host restatement of spmm_xbsr_reblock32_nnzb + spmm_sbsr_reblock32: block
    (I, J) of size bs into block (I // R, J // R) of size 32 at sub-block
    (I % R, J % R), R = 32 // bs, the rest zero; direction kept."""
    R = 32 // bs
    mb32 = -(-mb // R)
    vb = v.reshape(-1, bs, bs)
    rows32, vals = [], {}
    for I32 in range(mb32):
        cols = set()
        for I in range(I32 * R, min(mb, I32 * R + R)):
            for k in range(rp[I], rp[I + 1]):
                J = int(ci[k])
                cols.add(J // R)
                blk = vals.setdefault((I32, J // R), np.zeros((32, 32), np.float32))
                r0, c0 = (I % R) * bs, (J % R) * bs
                if direction == 0:
                    blk[r0:r0 + bs, c0:c0 + bs] = vb[k]
                else:  # COLUMN blocks: stored transposed, and so is the 32 x 32 block
                    blk[c0:c0 + bs, r0:r0 + bs] = vb[k]
        rows32.append(sorted(cols))
    rp32 = np.concatenate([[0], np.cumsum([len(c) for c in rows32])]).astype(np.int32)
    ci32 = np.array([c for cs in rows32 for c in cs], np.int32)
    v32 = np.stack([vals[(I32, c)] for I32, cs in enumerate(rows32) for c in cs]) \
        if ci32.size else np.zeros((0, 32, 32), np.float32)
    return rp32, ci32, v32.reshape(-1)


@pytest.mark.parametrize("bs", [2, 4, 8, 16])
@pytest.mark.parametrize("direction", [0, 1])
def test_bsr_reblock32_exact_and_product(oracle, device, bs, direction):
    """spmm_xbsr_reblock32_nnzb + spmm_sbsr_reblock32 against the host
    restatement, bit for bit (row pointer, block columns, every value and
    zero), for ROW and COLUMN blocks, an mb the ratio R = 32 / bs does not
    divide and an empty block row; then the bs 32 analysed stream on the
    re-blocked matrix against the f64 oracle of the ORIGINAL matrix."""
    from spmm_hip._lib import DIRECTION_COLUMN, DIRECTION_ROW
    ops = _ops()
    rng = np.random.default_rng(40 + bs + 7 * direction)
    R = 32 // bs
    mb, kb = 5 * R + 3, 4 * R + 1
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, 0.15, empty_rows=(2,))
    dr = DIRECTION_ROW if direction == 0 else DIRECTION_COLUMN
    drp, dci, dv = _dev(rp, ci, v)
    rp32, ci32, v32 = ops.bsr_reblock32(drp, dci, dv, mb=mb, bs=bs, direction=dr)
    torch.cuda.synchronize()
    wrp, wci, wv = _reblock32_numpy(rp, ci, v, bs, mb, direction)
    assert np.array_equal(rp32.cpu().numpy(), wrp)
    assert np.array_equal(ci32.cpu().numpy(), wci)
    assert np.array_equal(v32.cpu().numpy(), wv), "values placed differently"
    mb32, kb32 = -(-mb // R), -(-kb // R)
    n = 128
    Bh = np.zeros((kb32 * 32, n), np.float32)
    Bh[:kb * bs] = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    if direction == 0:
        masks, vcol = ops.bsr32_analysis(v32, nnzb=int(ci32.numel()))
        C = torch.zeros((mb32 * 32, n), device=device)
        ops.bsrmm_analysed(rp32, ci32, vcol, masks, torch.from_numpy(Bh).to(device), mb=mb32,
                           kb=kb32, n=n, ldb=n, C=C, ldc=n)
    else:
        C = torch.zeros((mb32 * 32, n), device=device)
        ops.bsrmm(rp32, ci32, v32, torch.from_numpy(Bh).to(device), mb=mb32, kb=kb32, n=n, bs=32,
                  ldb=n, C=C, ldc=n, direction=dr)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, direction, mb, n, bs, rp, ci, v, Bh[:kb * bs], n, 0)
    got = C.cpu().numpy()
    assert_normwise(got[:mb * bs], ref, absd, TOL_F32, f"reblocked bs {bs} dir {direction}")
    assert not got[mb * bs:].any(), "rows past mb * bs must stay zero"


def test_bsr_reblock32_matches_csr2bsr32_full_size(device):
    """At full size (the reddit stand-in): csr2bsr at bs 8 then re-blocking to
    32 is, bit for bit, csr2bsr at bs 32 of the same CSR (the same blocks, the
    same values, the same explicit zeros)."""
    from spmm_hip import prep
    ops = _ops()
    n = 232965
    rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    b8 = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=8)
    b32 = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=32)
    del dci, dv
    mb8 = (n + 7) // 8
    r32 = ops.bsr_reblock32(b8[0], b8[1], b8[2], mb=mb8, bs=8)
    torch.cuda.synchronize()
    assert torch.equal(r32[0], b32[0]) and torch.equal(r32[1], b32[1])
    assert torch.equal(r32[2], b32[2]), "re-blocked values differ from csr2bsr at bs 32"


def _grouped_items(rp, ci, v, bs, W, mb):
    """Items of the group analysis restated on the host (test_group_analysis_layout's
    grouping): per group of W block rows, the union of their blocks' nonzero
    columns cut into items of 16 (bs 16)."""
    E = 16 if bs == 16 else 8
    vb = v.astype(np.float32).reshape(-1, bs, bs)
    nz = [np.nonzero((np.abs(vb[k]) > 0).any(axis=0))[0] for k in range(vb.shape[0])]
    items = 0
    for g in range(-(-mb // W)):
        ent = set()
        for br in range(g * W, min(mb, g * W + W)):
            for k in range(rp[br], rp[br + 1]):
                ent.update(int(ci[k]) * bs + int(c) for c in nz[k])
        items += -(-len(ent) // E)
    return items


def _auto_group_rows(oracle, device, shared):
    """groupRows = 0 at bs 16: the library analyses W = 2, 4 and 8 and keeps the
    least items(W) * (2.74 + W) (group.cpp's model). The choice must be that
    minimum over the host restatement of the items, the buffer must equal an
    explicit analysis with that W byte for byte (its header word 0 holds W),
    and the product must match the oracle. Returns the choice."""
    ops = _ops()
    rng = np.random.default_rng(5 + shared)
    mb, kb = 48, 96
    rows = []
    for br in range(mb):
        if shared:  # a band of block columns around the diagonal: neighbours share most
            c = np.arange(max(0, br - 3), min(kb, br + 4))
        else:       # every block row its own two columns
            c = np.array([(2 * br) % kb, (2 * br + 1) % kb])
        rows.append(np.sort(c))
    rp = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1] * 256).astype(np.float16)
    cost = {W: _grouped_items(rp, ci, v, 16, W, mb) * (2.74 + W) for W in (2, 4, 8)}
    want = min(cost, key=lambda W: (cost[W], W))
    drp, dci, dv = _dev(rp, ci, v)
    auto = ops.GroupedBsr16(drp, dci, dv, mb=mb, group_rows=0)
    assert auto.W == want, (auto.W, cost)
    manual = ops.GroupedBsr16(drp, dci, dv, mb=mb, group_rows=want)
    assert manual.W == want and torch.equal(auto.buffer, manual.buffer)
    n = 256
    Bh = rng.uniform(-1, 1, (kb * 16, n)).astype(np.float16)
    C = torch.zeros((mb * 16, n), device=device)
    auto.mm(torch.from_numpy(Bh).to(device), kb=kb, n=n, ldb=n, C=C, ldc=n)
    torch.cuda.synchronize()
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, 16, rp, ci, v, Bh, n, 0, half=True)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F16_ACC, f"auto W={auto.W}")
    auto.close()
    manual.close()
    return want


def test_group_rows_chosen_by_the_library(oracle, device):
    """Neighbouring block rows sharing most columns (a banded pattern) and
    sharing none pick different W through _auto_group_rows: more rows per group
    where they share."""
    ws = [_auto_group_rows(oracle, device, s) for s in (True, False)]
    assert ws == [4, 2], ws


@pytest.mark.parametrize("seed", range(20))
def test_random_shapes_bits(oracle, device, seed):
    """Random BSR matrices (empty block rows, all-zero blocks and columns, rows of
    0 .. 60 blocks), bs 2 / 4 / 8 / 32 / 64, n from 4 to 256, random alpha / beta:
    the entries that share a stream's arithmetic give the same bits, signed zeros
    included, and those DESIGN.md §6 calls bit-exact equal the sequential fp32
    oracle bit for bit (bs 2 / 4 / 8 on both kernels, bs 32 / 64 on the column
    stream at row-major C); bs 32: the drop-in, analysed and grouped entries are
    bit-identical."""
    from spmm_hip._lib import BSR_SMALL_GROUPED
    ops = _ops()
    rng = np.random.default_rng(9100 + seed)
    bs = int(rng.choice([2, 4, 8, 32, 64]))
    n = int(rng.choice([4, 8, 36, 64, 96, 128, 132, 256]))
    mb = int(rng.integers(1, 120 if bs >= 32 else 900))
    kb = int(rng.integers(1, 200 if bs >= 32 else 2000))
    p = float(rng.choice([0.02, 0.1, 0.3]))
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, p, empty_rows=tuple(rng.choice(mb, min(3, mb), replace=False)))
    vb = v.reshape(-1, bs, bs)
    nnzb = vb.shape[0]
    if nnzb:
        vb[rng.random(nnzb) < 0.2] = 0.0                                    # all-zero blocks
        vb[:, :, :][rng.random((nnzb, 1, bs)).repeat(bs, axis=1) < 0.4] = 0.0  # zero columns
        vb[rng.random((nnzb, bs, bs)) < 0.3] = 0.0                           # explicit zeros
    v = vb.reshape(-1)
    alpha = float(rng.choice([1.0, -0.5, 2.0]))
    beta = float(rng.choice([0.0, 0.0, 0.75]))
    B = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (mb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    what = f"bs={bs} n={n} mb={mb} kb={kb} nnzb={nnzb} alpha={alpha} beta={beta}"

    def run(flags=0, **kw):
        h = ops.Handle()
        h.set_bsr_options(flags)
        C = torch.from_numpy(C0.copy()).to(device)
        ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C, ldc=n, alpha=alpha,
                  beta=beta, handle=h, **kw)
        torch.cuda.synchronize()
        h.close()
        return C

    C = run()
    if nnzb == 0:  # rocsparse_bsrmm.h:152-154's quick return: C untouched, beta or not
        assert torch.equal(run().view(torch.int32), torch.from_numpy(C0).to(device).view(torch.int32))
        return
    ref = oracle_bsrmm_f32(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0, alpha=alpha, beta=beta,
                           C=C0.reshape(-1)).reshape(mb * bs, n)
    ref64, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    ref64 = alpha * ref64 + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    got = C.cpu().numpy()
    assert_normwise(got, ref64, absd, TOL_F32, what)
    bits = lambda t: (t.view(torch.int32) if isinstance(t, torch.Tensor) else t.view(np.int32))
    # block rows the column stream may cut into segments on a shallow grid (longer than 64
    # blocks, bsr_kernels.hip cs2_segments) sum their partials in segment order
    whole = np.repeat(np.diff(rp) <= 64, bs) if bs >= 32 else np.ones(mb * bs, bool)
    assert np.array_equal(got[whole], ref[whole]), what + ": not the sequential fp32 chain"
    bad = bits(got[whole]) != bits(ref[whole])
    assert not bad.any(), f"{what}: {int(bad.sum())} signed zeros differ from the oracle"
    wt = torch.from_numpy(whole).to(device)
    if bs <= 8:
        Cg = run(BSR_SMALL_GROUPED)
        assert torch.equal(bits(Cg), bits(C)), what + ": grouped stream differs from the default"
    if bs == 32:
        masks, vcol = ops.bsr32_analysis(dv, nnzb=nnzb)
        Ca = torch.from_numpy(C0.copy()).to(device)
        ops.bsrmm_analysed(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=Ca, ldc=n,
                           alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        assert torch.equal(bits(Ca), bits(C)), what + ": analysed entry differs"
        if n % 4 == 0:
            grp = ops.GroupedBsr32(drp, dci, dv, mb=mb)
            Cg = torch.from_numpy(C0.copy()).to(device)
            grp.mm(dB, kb=kb, n=n, ldb=n, C=Cg, ldc=n, alpha=alpha, beta=beta)
            torch.cuda.synchronize()
            assert torch.equal(bits(Cg[wt]), bits(C[wt])), what + ": grouped entry differs"
            grp.close()


@pytest.mark.parametrize("seed", range(10))
def test_random_shapes_bs16_f16_bits(oracle, device, seed):
    """bs 16 fp16 (config 5's types) on random matrices with empty block rows and zero
    blocks / columns, n 16 to 512: the drop-in and analysed entries give the same bits,
    signed zeros included; both are within the fp16-input bar of the exact product, and
    so is the grouped entry (W by the library)."""
    ops = _ops()
    rng = np.random.default_rng(9300 + seed)
    bs = 16
    n = int(rng.choice([16, 64, 128, 256, 264, 512]))
    mb = int(rng.integers(1, 400))
    kb = int(rng.integers(1, 600))
    p = float(rng.choice([0.01, 0.05, 0.2]))
    rp, ci, v = _rand_bsr(rng, mb, kb, bs, p, empty_rows=tuple(rng.choice(mb, min(3, mb), replace=False)))
    vb = v.reshape(-1, bs, bs)
    nnzb = vb.shape[0]
    if nnzb:
        vb[rng.random(nnzb) < 0.2] = 0.0
        vb[rng.random((nnzb, 1, bs)).repeat(bs, axis=1) < 0.5] = 0.0
    v16 = vb.reshape(-1).astype(np.float16)
    alpha = float(rng.choice([1.0, -0.5]))
    beta = float(rng.choice([0.0, 0.5]))
    B16 = rng.uniform(-1, 1, (kb * bs, n)).astype(np.float16)
    C0 = rng.uniform(-1, 1, (mb * bs, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v16, B16)
    what = f"bs16 fp16 n={n} mb={mb} kb={kb} nnzb={nnzb} alpha={alpha} beta={beta}"
    C1 = torch.from_numpy(C0.copy()).to(device)
    ops.bsrmm_f16(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=n, alpha=alpha,
                  beta=beta)
    masks, vcol = ops.bsr16_analysis(dv, nnzb=nnzb)
    C2 = torch.from_numpy(C0.copy()).to(device)
    ops.bsrmm_analysed_f16(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=C2, ldc=n,
                           alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    assert torch.equal(C1.view(torch.int32), C2.view(torch.int32)), what + ": analysed differs"
    if nnzb == 0:  # rocsparse_bsrmm.h:152-154's quick return: C untouched
        assert np.array_equal(C1.cpu().numpy().view(np.int32), C0.view(np.int32))
        return
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v16.astype(np.float32),
                                 B16.astype(np.float32), n, 0)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(C1.cpu().numpy(), ref, absd, TOL_F16_ACC, what)
    if n % 8 == 0:
        grp = ops.GroupedBsr16(drp, dci, dv, mb=mb)
        C3 = torch.from_numpy(C0.copy()).to(device)
        grp.mm(dB, kb=kb, n=n, ldb=n, C=C3, ldc=n, alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        assert_normwise(C3.cpu().numpy(), ref, absd, TOL_F16_ACC, what + " grouped")
        grp.close()


@pytest.mark.parametrize("layout,n", [("row", 64), ("row", 128), ("col", 64), ("col", 132)])
@pytest.mark.parametrize("fill", ["dense", "mostly", "sparse"])
def test_panel_stream_bits(oracle, device, layout, n, fill):
    """The bs 32 panel stream (bsr32_f32_panel_kernel, round 6): from 2^15 blocks the drop-in
    call probes the blocks' nonzero columns and, when they hold at least 24 of 32 on average,
    runs the panel stream instead of the column stream. Both issue the same fused
    multiply-adds per output in the same order and skip the same all-zero columns, so the
    drop-in's bits equal the analysed entry's (the column stream on the analysis's masks) for
    dense blocks (the reference sweep's), blocks with 4 zero columns each and zero blocks
    (mostly), and column-sparse blocks (the column stream itself); both C layouts, the 64-
    and 128-column tiles, alpha / beta on the column-major form; against the f64 oracle on
    one case."""
    ops = _ops()
    rng = np.random.default_rng(7300 + n + {"dense": 0, "mostly": 1, "sparse": 2}[fill])
    # rows of at most 64 blocks: a shallow grid cuts longer rows of a row-major C into segments
    # (column stream, cs2_segments), which the panel stream leaves to the column stream
    mb, kb, bs = 560, 256, 32
    per_row = 60
    ci = np.concatenate([np.sort(rng.choice(kb, per_row, replace=False)) for _ in range(mb)])
    rp = np.arange(0, mb * per_row + 1, per_row, dtype=np.int32)
    nnzb = ci.size
    assert nnzb >= 1 << 15
    vb = rng.uniform(-1, 1, (nnzb, bs, bs)).astype(np.float32)
    if fill != "dense":
        zc = 4 if fill == "mostly" else 20
        cols = np.argsort(rng.random((nnzb, bs)), axis=1)[:, :zc]
        vb[np.arange(nnzb)[:, None, None], np.arange(bs)[None, :, None], cols[:, None, :]] = 0.0
        vb[rng.random(nnzb) < 0.01] = 0.0
    v = vb.reshape(-1)
    m, k = mb * bs, kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = (1.0, 0.0) if layout == "row" else (0.5, -1.5)
    drp, dci, dv, dB = _dev(rp, ci.astype(np.int32), v, B.reshape(-1))
    ld, oc = (n, ops.ORDER_ROW) if layout == "row" else (m, ops.ORDER_COL)

    def fresh():
        c = C0 if layout == "row" else np.ascontiguousarray(C0.T)
        return torch.from_numpy(c.reshape(-1).copy()).cuda()

    def host(t):
        a = t.cpu().numpy()
        return a.reshape(m, n) if layout == "row" else a.reshape(n, m).T

    C1 = fresh()
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=ld, order_c=oc,
              alpha=alpha, beta=beta)
    masks, vcol = ops.bsr32_analysis(dv, nnzb=nnzb)
    C2 = fresh()
    ops.bsrmm_analysed(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=C2, ldc=ld,
                       order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got, ref2 = host(C1), host(C2)
    diff = got.view(np.uint32) != ref2.view(np.uint32)
    assert not diff.any(), f"{fill} {layout} n={n}: {int(diff.sum())} elements differ in bits"
    if fill == "mostly" and layout == "row" and n == 128:
        ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
        assert_normwise(got, ref, absd, TOL_F32, "panel stream")


@pytest.mark.parametrize("layout,n", [("row", 64), ("row", 128), ("col", 128)])
@pytest.mark.parametrize("fill", ["dense", "mostly"])
def test_panel_stream_bs64_bits(device, layout, n, fill):
    """bs 64 runs the bs 32 streams over its 32 x 32 sub-blocks; from 2^15 sub-blocks the
    panel stream takes them when they are dense. Its bits equal the analysed bs 32 entry's
    (the column stream) on the same matrix re-blocked to bs 32."""
    ops = _ops()
    rng = np.random.default_rng(7400 + n + (fill == "mostly"))
    # 32 blocks per row: the bs 32 form's rows hold 64 sub-blocks, uncut (see above)
    mb, kb, bs = 256, 128, 64
    per_row = 32
    ci = np.concatenate([np.sort(rng.choice(kb, per_row, replace=False)) for _ in range(mb)])
    rp = np.arange(0, mb * per_row + 1, per_row, dtype=np.int32)
    nnzb = ci.size
    assert 4 * nnzb >= 1 << 15
    vb = rng.uniform(-1, 1, (nnzb, bs, bs)).astype(np.float32)
    if fill == "mostly":
        cols = np.argsort(rng.random((nnzb, bs)), axis=1)[:, :8]
        vb[np.arange(nnzb)[:, None, None], np.arange(bs)[None, :, None], cols[:, None, :]] = 0.0
    # the same matrix as bs 32: block row 2R + h holds (2C, 2C + 1) for each block (R, C)
    sub = vb.reshape(mb, per_row, 2, 32, 2, 32).transpose(0, 2, 1, 4, 3, 5)  # R, h, b, ch, 32, 32
    v32 = np.ascontiguousarray(sub).reshape(-1)
    ci32 = np.repeat(2 * ci.reshape(mb, 1, per_row), 2, axis=1)[..., None] + np.arange(2)
    ci32 = ci32.reshape(-1).astype(np.int32)
    rp32 = np.arange(0, 2 * mb * 2 * per_row + 1, 2 * per_row, dtype=np.int32)
    m, k = mb * bs, kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    alpha, beta = (1.0, 0.0) if layout == "row" else (0.5, -1.5)
    ld, oc = (n, ops.ORDER_ROW) if layout == "row" else (m, ops.ORDER_COL)

    def fresh():
        c = C0 if layout == "row" else np.ascontiguousarray(C0.T)
        return torch.from_numpy(c.reshape(-1).copy()).cuda()

    def host(t):
        a = t.cpu().numpy()
        return a.reshape(m, n) if layout == "row" else a.reshape(n, m).T

    drp, dci, dv, dB = _dev(rp, ci.astype(np.int32), vb.reshape(-1), B.reshape(-1))
    C1 = fresh()
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=ld, order_c=oc,
              alpha=alpha, beta=beta)
    del dv
    drp2, dci2, dv2 = _dev(rp32, ci32, v32)
    masks, vcol = ops.bsr32_analysis(dv2, nnzb=ci32.size)
    C2 = fresh()
    ops.bsrmm_analysed(drp2, dci2, vcol, masks, dB, mb=2 * mb, kb=2 * kb, n=n, ldb=n, C=C2,
                       ldc=ld, order_c=oc, alpha=alpha, beta=beta)
    torch.cuda.synchronize()
    got, ref = host(C1), host(C2)
    diff = got.view(np.uint32) != ref.view(np.uint32)
    assert not diff.any(), f"bs 64 {fill} {layout} n={n}: {int(diff.sum())} elements differ"


def test_panel_stream_edges(device):
    """The panel stream with row-major C and alpha / beta, a partial second column tile
    (n = 132), empty block rows and all-zero blocks among dense ones: bits equal the
    analysed column stream's."""
    ops = _ops()
    rng = np.random.default_rng(7500)
    mb, kb, bs, n, per_row = 700, 256, 32, 132, 60
    rows = [np.sort(rng.choice(kb, per_row, replace=False)) if r % 7 else np.zeros(0, int)
            for r in range(mb)]
    rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    nnzb = ci.size
    assert nnzb >= 1 << 15
    vb = rng.uniform(-1, 1, (nnzb, bs, bs)).astype(np.float32)
    vb[rng.random(nnzb) < 0.02] = 0.0
    m, k = mb * bs, kb * bs
    B = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, n)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, vb.reshape(-1), B.reshape(-1))
    C1 = torch.from_numpy(C0.reshape(-1).copy()).cuda()
    ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=kb, n=n, bs=bs, ldb=n, C=C1, ldc=n, alpha=-0.75,
              beta=1.25)
    masks, vcol = ops.bsr32_analysis(dv, nnzb=nnzb)
    C2 = torch.from_numpy(C0.reshape(-1).copy()).cuda()
    ops.bsrmm_analysed(drp, dci, vcol, masks, dB, mb=mb, kb=kb, n=n, ldb=n, C=C2, ldc=n,
                       alpha=-0.75, beta=1.25)
    torch.cuda.synchronize()
    assert torch.equal(C1.view(torch.int32), C2.view(torch.int32))
