"""Hot-column cache hints for the CSR gathers (spmm_csr_hot_analysis +
spmm_csrmm_hot_f32).

The analysis is pinned against its numpy restatement (column counts, the
count histogram with an open-ended top bin, the largest set of top-count
columns whose B-row pieces fit the byte budget). The product must equal the
plain csrmm on the untagged indices bit for bit (the tags change cache
policy only, never the arithmetic or its order), and the oracle within the
fp32 bar (gespmm_csrmm.h:124-129 semantics, as tests/test_gpu_csr.py)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from helpers import TOL_F32, assert_normwise, oracle_csrmm_f64

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HOT_BINS = 8192


def _ops():
    from spmm_hip import ops
    return ops


def _expected_tags(ci, k, base, hot_rows):
    """Restatement of the analysis: hot iff min(count, 8191) >= thr, thr the
    smallest bin whose suffix of columns fits in hot_rows."""
    cnt = np.bincount(ci.astype(np.int64) - base, minlength=k)
    clamp = np.minimum(cnt, HOT_BINS - 1)
    hist = np.bincount(clamp, minlength=HOT_BINS)
    suffix = np.concatenate([np.cumsum(hist[::-1])[::-1], [0]])
    thr = int(np.nonzero(suffix <= hot_rows)[0][0])
    return clamp[ci.astype(np.int64) - base] >= thr, thr


def _piece_bytes(n):
    tile = 256 if n > 128 else (128 if n > 64 else 64)
    return 4 * (n if n < tile else tile)


@pytest.mark.parametrize("base", [0, 1])
@pytest.mark.parametrize("hot_rows", [0, 1, 37, 500, 4000, 10 ** 7])
def test_analysis_matches_restatement(device, base, hot_rows):
    from spmm_hip import prep
    ops = _ops()
    rp, ci = prep.powerlaw_csr(20000, 400000, 9000, 2.3, 77)
    k = rp.size - 1
    ci_b = (ci + base).astype(np.int32)
    n = 128
    hb = hot_rows * _piece_bytes(n) if hot_rows else 4
    got = ops.csr_hot_analysis(torch.from_numpy(ci_b).to(device), n=n, k=k, base=base,
                               hot_bytes=hb).cpu().numpy()
    assert np.array_equal(got & 0x7fffffff, ci_b), "analysis changed an index"
    want, thr = _expected_tags(ci_b, k, base, hot_rows)
    assert np.array_equal(got < 0, want), f"tags differ (thr {thr})"
    hot_cols = np.unique(ci_b[want])
    assert hot_cols.size <= max(hot_rows, 0) or thr == 0


def test_analysis_open_top_bin_and_default(device):
    """Columns past the last count bin (>= 8191 nonzeros) share it: a budget
    below their number tags none of them; the default budget (hotBytes = 0)
    is SPMM_CSR_HOT_BYTES_DEFAULT."""
    ops = _ops()
    k = 64
    ci = np.concatenate([np.full(9000, c, np.int32) for c in range(3)] +
                        [np.arange(k, dtype=np.int32)])
    d = torch.from_numpy(ci).to(device)
    got = ops.csr_hot_analysis(d, n=128, k=k, hot_bytes=2 * 512).cpu().numpy()
    assert not (got < 0).any()
    got = ops.csr_hot_analysis(d, n=128, k=k, hot_bytes=3 * 512).cpu().numpy()
    assert np.array_equal(got < 0, ci < 3)
    got = ops.csr_hot_analysis(d, n=128, k=k, hot_bytes=0).cpu().numpy()
    assert (got < 0).all()  # 64 columns fit the 128-MB default


@pytest.mark.parametrize("K", [8, 32, 64, 100, 128, 256, 300])
@pytest.mark.parametrize("alpha,beta,orders", [(1.0, 0.0, (0, 0)), (0.5, 1.5, (0, 0)),
                                               (1.0, 0.0, (1, 1)), (2.0, -1.0, (0, 1))])
def test_hot_product_bit_identical(oracle, device, K, alpha, beta, orders):
    from spmm_hip import prep
    ops = _ops()
    rp, ci = prep.powerlaw_csr(6000, 90000, 3000, 2.3, 5)
    m = k = rp.size - 1
    rng = np.random.default_rng(K)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    Bn = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (m, K)).astype(np.float32)
    d_rp, d_ci, d_v = (torch.from_numpy(a).to(device) for a in (rp, ci, v))
    ob, oc = orders
    B = torch.from_numpy(np.ascontiguousarray(Bn.T if ob else Bn)).to(device)
    ldb = k if ob else K
    ldc = m if oc else K
    tag = ops.csr_hot_analysis(d_ci, n=K, k=k, hot_bytes=400 * _piece_bytes(K))
    assert 0 < int((tag < 0).sum()) < ci.size  # both policies are exercised

    def run(f, colind):
        C = torch.from_numpy(np.ascontiguousarray(C0.T if oc else C0)).to(device)
        f(d_rp, colind, d_v, B, n=K, k=k, ldb=ldb, order_b=ob, C=C, ldc=ldc, order_c=oc,
          alpha=alpha, beta=beta)
        torch.cuda.synchronize()
        c = C.cpu().numpy()
        return c.T if oc else c

    plain = run(ops.csrmm, d_ci)
    hot = run(ops.csrmm_hot, tag)
    assert np.array_equal(hot, plain), "hot-tagged product differs from the plain kernel"
    ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, Bn, K, 0)
    ref = alpha * ref + beta * C0.astype(np.float64)
    absd = abs(alpha) * absd + abs(beta) * np.abs(C0.astype(np.float64))
    assert_normwise(hot, ref, absd, TOL_F32, f"hot csrmm K={K} vs f64 oracle")


def test_hot_index_base_one(oracle, device):
    from spmm_hip import prep
    ops = _ops()
    rp, ci = prep.powerlaw_csr(3000, 40000, 1500, 2.3, 9)
    m = k = rp.size - 1
    K = 128
    rng = np.random.default_rng(3)
    v = rng.uniform(-1, 1, ci.size).astype(np.float32)
    Bn = rng.uniform(-1, 1, (k, K)).astype(np.float32)
    d_rp1 = torch.from_numpy(rp + 1).to(device)
    d_ci1 = torch.from_numpy(ci + 1).to(device)
    d_v, B = torch.from_numpy(v).to(device), torch.from_numpy(Bn).to(device)
    tag = ops.csr_hot_analysis(d_ci1, n=K, k=k, base=1, hot_bytes=200 * 512)
    C = torch.empty((m, K), device=device)
    ops.csrmm_hot(d_rp1, tag, d_v, B, n=K, k=k, ldb=K, C=C, ldc=K, base=1)
    C1 = torch.empty((m, K), device=device)
    ops.csrmm(d_rp1, d_ci1, d_v, B, n=K, k=k, ldb=K, C=C1, ldc=K, base=1)
    torch.cuda.synchronize()
    assert torch.equal(C, C1)
    ref, absd = oracle_csrmm_f64(oracle, m, K, rp, ci, v, Bn, K, 0)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F32, "hot csrmm base 1")


def test_hot_products_scale_bit_identical(device):
    """BASELINE's workload (products stand-in, K = 128) with the default
    budget: the hot product equals the plain kernel's C bit for bit."""
    from spmm_hip import prep
    ops = _ops()
    rp, ci = prep.powerlaw_csr(2449029, 61859140, 17481, 2.3, 1234)
    n, K = rp.size - 1, 128
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    d_rp, d_ci, d_v = (torch.from_numpy(a).to(device) for a in (rp, ci, v))
    g = torch.Generator(device=device)
    g.manual_seed(1234)
    B = torch.rand((n, K), device=device, generator=g) * 2 - 1
    tag = ops.csr_hot_analysis(d_ci, n=K, k=n)
    frac = float((tag < 0).float().mean())
    assert 0.3 < frac < 0.9, f"hot share of the gathers {frac}"
    C1 = torch.empty((n, K), device=device)
    C2 = torch.empty((n, K), device=device)
    ops.csrmm(d_rp, d_ci, d_v, B, n=K, k=n, ldb=K, C=C1, ldc=K)
    ops.csrmm_hot(d_rp, tag, d_v, B, n=K, k=n, ldb=K, C=C2, ldc=K)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)


def test_hot_status_codes(device):
    from spmm_hip._lib import INVALID_VALUE, NOT_INITIALIZED, lib
    L = lib()
    h = _ops().default_handle()
    ci = torch.zeros(4, dtype=torch.int32, device=device)
    out = torch.empty_like(ci)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert L.spmm_csr_hot_analysis(None, 8, 4, 4, p(ci), 0, 0, p(out)) == NOT_INITIALIZED
    assert L.spmm_csr_hot_analysis(h.raw, 8, 4, 4, p(ci), 0, -1, p(out)) == INVALID_VALUE
    assert L.spmm_csr_hot_analysis(h.raw, 8, 4, 4, p(ci), 2, 0, p(out)) == INVALID_VALUE
    assert L.spmm_csr_hot_analysis(h.raw, 8, 4, 4, None, 0, 0, p(out)) == INVALID_VALUE
    assert L.spmm_csr_hot_analysis(h.raw, 8, 4, 0, None, 0, 0, None) == 0
    assert L.spmm_csrmm_hot_f32(None, 1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0,
                                None, 1, 0) == NOT_INITIALIZED
    assert L.spmm_csrmm_hot_f32(h.raw, -1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0,
                                None, 1, 0) == INVALID_VALUE


def test_hot_per_row_resource_beyond_4gb(device):
    """B whose row offsets pass 4 GB (k * ldb * 4 > 2^32): the kernel then builds a
    buffer resource per row (HOT = 1) instead of one for all of B with the row in
    soffset (HOT = 2). Bit-identical to the plain kernel; fp64 reference on the GPU."""
    ops = _ops()
    m, k, n, ldb, nnz = 20000, 1_100_000, 128, 1024, 200_000
    g = torch.Generator(device=device)
    g.manual_seed(7)
    B = torch.rand((k, ldb), device=device, generator=g) * 2 - 1  # 4.5 GB
    rows = torch.sort(torch.randint(0, m, (nnz,), device=device, generator=g)).values
    ci = torch.randint(0, k, (nnz,), device=device, generator=g, dtype=torch.int32)
    ci[:50] = k - 1  # the last rows of B, past the 4-GB offset
    rows[:50] = 0
    rows = torch.sort(rows).values
    rp = torch.zeros(m + 1, dtype=torch.int64, device=device)
    rp[1:] = torch.cumsum(torch.bincount(rows, minlength=m), 0)
    rp = rp.to(torch.int32)
    v = torch.rand(nnz, device=device, generator=g) * 2 - 1
    tag = ops.csr_hot_analysis(ci, n=n, k=k, hot_bytes=20000 * 512)
    assert 0 < int((tag < 0).sum()) < nnz
    C1 = torch.empty((m, n), device=device)
    C2 = torch.empty((m, n), device=device)
    ops.csrmm(rp, ci, v, B, n=n, k=k, ldb=ldb, C=C1, ldc=n)
    ops.csrmm_hot(rp, tag, v, B, n=n, k=k, ldb=ldb, C=C2, ldc=n)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)
    ref = torch.zeros((m, n), dtype=torch.float64, device=device)
    ref.index_add_(0, rows, v.double()[:, None] * B[ci.long(), :n].double())
    absd = torch.zeros_like(ref).index_add_(0, rows, (v.double()[:, None] *
                                                      B[ci.long(), :n].double()).abs())
    assert_normwise(C2.cpu().numpy(), ref.cpu().numpy(), absd.cpu().numpy(), TOL_F32,
                    "hot csrmm, B past 4 GB")
    del B
