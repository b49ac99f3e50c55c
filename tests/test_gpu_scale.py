"""Path B at BASELINE's full sizes.

Checks per result:
* every row against the f64 oracle of the whole product (_check_oracle_all,
  round 5: the oracle's nonzero-outer loop reads B rows contiguously, so the
  10^8-nonzero products check in seconds on the box's host cores);
* sampled rows against the f64 oracle (oracle_csrmm_f64 on the same CSR
  values the BSR / hybrid arrays were built from: the product is the same
  matrix's), as the reference's own differential bar does
  (check_result.cu:233-246): every row of the longest block row, of a
  segmented block row where the launch splits rows (seg_build_kernel), of the
  block rows launched first and last (XCD-chunked order, and longest-first on
  shallow grids), and 1,500 random rows;
* every row against the CSR kernel, an independent implementation of the
  same product, within the fp32 bar, with the magnitude bound |A|.|B|
  computed on the device (the CSR kernel on |val|, |B|).
The small-size tests pin each kernel to the oracle element by element; these
check that nothing breaks at 10^8 nonzeros (index widths, grid sizes, tails,
segments, launch orders)."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import TOL_F16_ACC, TOL_F32, assert_normwise, oracle_csrmm_f64

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ops():
    from spmm_hip import ops
    return ops


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _xcd_block_row(b: int, mb: int, xm: int = 32) -> int:
    """bsr_kernels.hip xcd_block_row: block row of wave b in the XCD-chunked order."""
    full = mb // (8 * xm) * (8 * xm)
    if b >= full:
        return b
    x, i = b % 8, b // 8
    return ((i // xm) * 8 + x) * xm + i % xm


def _sample_rows(brp: np.ndarray, bs: int, n: int, seed: int, extra_block_rows=()) -> np.ndarray:
    """Rows to check against the oracle: the longest and shortest block rows,
    the first and last block rows of the XCD-chunked launch order, any extra
    block rows (segmented ones), and 1,500 random rows."""
    nbr = np.diff(brp)
    mb = nbr.size
    brs = {int(np.argmax(nbr)), int(np.argmin(nbr)), 0, _xcd_block_row(mb - 1, mb), mb - 1}
    brs |= {int(b) for b in extra_block_rows}
    rows = [np.arange(b * bs, min((b + 1) * bs, n)) for b in sorted(brs)]
    rows.append(np.random.default_rng(seed).choice(n, 1500, replace=False))
    return np.unique(np.concatenate(rows))


def _segmented_block_rows(brp: np.ndarray, num_cus: int = 256) -> list[int]:
    """Block rows the bs = 32 launch cuts into segments (cs2_segments: a
    shallow grid whose longest row exceeds twice the mean load per wave slot;
    rows longer than L blocks are split): the shortest and the longest such."""
    nbr = np.diff(brp)
    nnzb, slots = int(nbr.sum()), 12 * num_cus
    if nbr.size > 8 * slots or nbr.max() <= 2 * (nnzb + slots - 1) // slots:
        return []
    L = max(64, (nnzb + 2 * slots - 1) // (2 * slots))
    seg = np.nonzero(nbr > L)[0]
    return [] if seg.size == 0 else [int(seg[np.argmin(nbr[seg])]), int(seg[np.argmax(nbr[seg])])]


def _check_oracle_rows(oracle, got, rp, ci, v, B, rows, tol, what):
    """got[rows] against the f64 oracle of the same rows of the CSR product;
    only the B rows those rows touch leave the device."""
    K = B.shape[1]
    deg = np.diff(rp)
    sub_rp = np.concatenate([[0], np.cumsum(deg[rows])]).astype(np.int32)
    sub_ci = np.concatenate([ci[rp[r]:rp[r + 1]] for r in rows])
    sub_v = np.concatenate([v[rp[r]:rp[r + 1]] for r in rows]).astype(np.float32)
    ucols, inv = np.unique(sub_ci, return_inverse=True)
    Bsub = B[torch.from_numpy(ucols.astype(np.int64)).to(B.device)].float().cpu().numpy()
    ref, absd = oracle_csrmm_f64(oracle, rows.size, K, sub_rp, inv.astype(np.int32), sub_v, Bsub,
                                 K, 0)
    g = got[torch.from_numpy(rows.astype(np.int64)).to(got.device)].cpu().numpy()
    assert_normwise(g, ref, absd, tol, f"{what}: {rows.size} sampled rows vs the f64 oracle")


def _check_oracle_all(oracle, got, rp, ci, v, B, tol, what):
    """Every row of got against the f64 oracle of the whole CSR product (B read
    row-major, contiguous per nonzero: seconds on the box's host cores)."""
    n = rp.size - 1
    K = B.shape[1]
    Bh = B.float().cpu().numpy()
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, Bh, K, 0)
    del Bh
    assert_normwise(got[:n].cpu().numpy(), ref, absd, tol, f"{what}: every row vs the f64 oracle")


def _within(got, ref, absd, tol, what):
    err = (got - ref).abs()
    bound = tol * absd + 1e-30
    bad = int((err > bound).sum())
    assert bad == 0, f"{what}: {bad} elements outside {tol} x |A||B| (max err {float(err.max())})"


def test_reddit_scale_bsr32_and_hybrid_vs_csr(oracle, device):
    """Config 3 (reddit stand-in, 115 M nnz, bs = 32, K = 128): device csr2bsr
    -> the column-stream MFMA kernel, and divide -> hybrid, each against
    sampled oracle rows and the CSR kernel."""
    from spmm_hip import prep
    ops = _ops()
    n, K, bs = 232965, 128, 32
    rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=device) * 2 - 1
    Cc = ops.gespmm_csrmm(drp, dci, dv, B[:n].contiguous())
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B[:n].abs().contiguous())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    assert int(bci.numel()) > 1_000_000
    # One run: the counted waits of the copy rings are checked on the emitted
    # code (tests/test_isa_waits.py), not by repetition.
    Cb = torch.empty((mb * bs, K), device=device)
    ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb, ldc=K)
    torch.cuda.synchronize()
    brp_h = brp.cpu().numpy()
    rows = _sample_rows(brp_h, bs, n, 11, _segmented_block_rows(brp_h))
    _check_oracle_rows(oracle, Cb, rp, ci, v, B, rows, TOL_F32, "reddit bs32 BSR")
    _check_oracle_all(oracle, Cb, rp, ci, v, B, TOL_F32, "reddit bs32 BSR")
    _within(Cb[:n], Cc, absd, 2 * TOL_F32, "reddit bs32 BSR vs CSR")
    assert not bool(Cb[n:].any()), "padding rows of C must be zero"
    del brp, bci, bval
    parts = prep.divide(n, rp, ci, v, bs, prep.hybrid_plan(rp, ci, bs, K)["density"])
    d = _dev(*parts)
    from spmm_hip._lib import HYBRID_SPLIT_BF16
    for flags in (0, HYBRID_SPLIT_BF16):
        h = ops.Handle()
        h.set_hybrid_options(flags)
        Ch = torch.empty((mb * bs, K), device=device)
        ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), B, m=n, n=K, k=n, bs=bs, ldb=K, C=Ch,
                         ldc=K, handle=h)
        torch.cuda.synchronize()
        _check_oracle_rows(oracle, Ch, rp, ci, v, B, _sample_rows(parts[3], bs, n, 12), TOL_F32,
                           f"reddit hybrid (flags {flags})")
        _within(Ch[:n], Cc, absd, 2 * TOL_F32, f"reddit hybrid (flags {flags}) vs CSR")
        h.close()


def test_products_scale_bsr16_f16_vs_csr(oracle, device):
    """Config 5 (products stand-in, bs = 16, fp16 A and B, K = 512): the
    fp16 MFMA kernel against sampled oracle rows (the exact product of the
    same fp16 values) and against the CSR kernel run on the same
    fp16-rounded values in fp32 (both accumulate in fp32)."""
    from spmm_hip import prep
    ops = _ops()
    n, K, bs = 2449029, 512, 16
    rp, ci = prep.community_csr(n, 27.0, 32, 512, 0.97, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float16).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B16 = (torch.rand((mb * bs, K), device=device) * 2 - 1).half()
    Bf = B16[:n].float().contiguous()
    Cc = ops.gespmm_csrmm(drp, dci, dv, Bf)
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), Bf.abs())
    del Bf
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    bval16 = bval.half()
    del bval
    Cb = torch.empty((mb * bs, K), device=device)
    ops.bsrmm_f16(brp, bci, bval16, B16, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb, ldc=K)
    torch.cuda.synchronize()
    assert int(bci.numel()) > 4_000_000
    rows = _sample_rows(brp.cpu().numpy(), bs, n, 13)
    _check_oracle_rows(oracle, Cb, rp, ci, v, B16, rows, TOL_F16_ACC, "products bs16 fp16 BSR")
    _check_oracle_all(oracle, Cb, rp, ci, v, B16, TOL_F16_ACC, "products bs16 fp16 BSR")
    _within(Cb[:n], Cc, absd, 2 * TOL_F16_ACC, "products bs16 fp16 BSR vs CSR")


@pytest.mark.parametrize("bs", [32, 16])
def test_reordered_reddit_scale_bsr_vs_csr(oracle, device, bs):
    """Configs 3 / 5 with the reorder step in the loop (reorder_graph.cc:26-49
    then run_bsrmm.cu): the reddit stand-in with scrambled node ids, the
    in-repo RCM (spmm_reorder_rcm), the permutation applied, device csr2bsr,
    the shipped bs kernel (bs 32 fp32, bs 16 fp16) against the CSR kernel on
    the same reordered matrix. RCM leaves far more, far emptier blocks than
    the generator's community order, so every ring and tail path of the
    column-stream / column-masked kernels is hit on a different block mix."""
    from spmm_hip import prep
    ops = _ops()
    n, K = 232965, 128
    rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    rp, ci = prep.permute_csr(rp, ci, np.random.default_rng(9).permutation(n).astype(np.int32))
    rp, ci = prep.permute_csr(rp, ci, prep.reorder(rp, ci, "rcm"))
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    if bs == 16:
        v = v.astype(np.float16).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=device) * 2 - 1
    if bs == 16:
        B = B.half().float()
    Cc = ops.gespmm_csrmm(drp, dci, dv, B[:n].contiguous())
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B[:n].abs().contiguous())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    assert int(bci.numel()) > (3_000_000 if bs == 32 else 5_000_000)
    Cb = torch.empty((mb * bs, K), device=device)
    if bs == 32:
        ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb, ldc=K)
        tol = 2 * TOL_F32
    else:
        ops.bsrmm_f16(brp, bci, bval.half(), B.half(), mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cb,
                      ldc=K)
        tol = 2 * TOL_F16_ACC
    torch.cuda.synchronize()
    brp_h = brp.cpu().numpy()
    seg = _segmented_block_rows(brp_h) if bs == 32 else []
    if bs == 32:
        assert seg, "the RCM-reordered reddit stand-in must exercise the segmented rows"
    rows = _sample_rows(brp_h, bs, n, 14 + bs, seg)
    _check_oracle_rows(oracle, Cb, rp, ci, v, B, rows, TOL_F32 if bs == 32 else TOL_F16_ACC,
                       f"RCM-reordered reddit bs{bs} BSR")
    _within(Cb[:n], Cc, absd, tol, f"RCM-reordered reddit bs{bs} BSR vs CSR")
    assert not bool(Cb[n:].any()), "padding rows of C must be zero"
    if bs == 32:
        # the hybrid on the same matrix: its remainder averages ~2,300 entries per
        # block row with heavy rows of ~17 k, the fused launch's longest-first order
        del brp, bci, bval, Cb
        parts = prep.divide(n, rp, ci, v, bs, prep.hybrid_plan(rp, ci, bs, K)["density"])
        d = _dev(*parts)
        Ch = torch.empty((mb * bs, K), device=device)
        ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), B, m=n, n=K, k=n, bs=bs, ldb=K, C=Ch, ldc=K)
        torch.cuda.synchronize()
        _check_oracle_rows(oracle, Ch, rp, ci, v, B, _sample_rows(parts[3], bs, n, 15), TOL_F32,
                           "RCM-reordered reddit hybrid")
        _within(Ch[:n], Cc, absd, 2 * TOL_F32, "RCM-reordered reddit hybrid vs CSR")


# ---------------------------------------------------------------------------
# The analysed entries at full size (spmm_bsr32_analysis_f32 +
# spmm_bsrmm_analysed_f32, spmm_bsr16_analysis_f16 + spmm_bsrmm_analysed_f16):
# the entries north_star's MFMA claim rests on, on the same stand-ins as the
# drop-in tests above, with the same two checks, plus bit-identity with the
# drop-in column stream on the same matrix (same items, order and segments).
# ---------------------------------------------------------------------------
def _graph(kind: str, reorder: bool):
    """(rp, ci, n) of the reddit / products community stand-ins (bench.py
    WORKLOADS), optionally with ids scrambled and the in-repo RCM applied."""
    from spmm_hip import prep
    if kind == "reddit":
        n = 232965
        rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    else:
        n = 2449029
        rp, ci = prep.community_csr(n, 27.0, 32, 512, 0.97, 1234)
    if reorder:
        rp, ci = prep.permute_csr(rp, ci, np.random.default_rng(9).permutation(n).astype(np.int32))
        rp, ci = prep.permute_csr(rp, ci, prep.reorder(rp, ci, "rcm"))
    return rp, ci, n


@pytest.mark.parametrize("kind,reorder", [("reddit", False), ("reddit", True),
                                          ("products", False), ("products", True)])
def test_analysed_bs32_full_size(oracle, device, kind, reorder):
    """Config 3's bs 32 fp32 product on the analysed entry at full size:
    reddit (1.8 M blocks), reddit after RCM (segmented outlier rows: the
    segment partials and their fix-up), products (2.96 M blocks: the
    column-major copy valCol is 12 GB, past 2^31 bytes, so every 64-bit block
    offset is exercised) and products after RCM (10.5 M blocks, 43 GB of
    valCol). Sampled rows against the f64 oracle (check_result.cu:233-246's
    bar is 1e-5 relative here), every row against the CSR kernel, and C
    bit-identical to the drop-in column stream on the same blocks."""
    ops = _ops()
    rp, ci, n = _graph(kind, reorder)
    K, bs = 128, 32
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=device) * 2 - 1
    Cc = ops.gespmm_csrmm(drp, dci, dv, B[:n].contiguous())
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B[:n].abs().contiguous())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    del dci, dv
    nnzb = int(bci.numel())
    Cd = torch.empty((mb * bs, K), device=device)
    ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cd, ldc=K)
    masks, vcol = ops.bsr32_analysis(bval, nnzb=nnzb)
    del bval
    if kind == "products":
        assert vcol.numel() * 4 > 2 ** 31, "valCol must pass 2^31 bytes"
    Ca = torch.empty((mb * bs, K), device=device)
    ops.bsrmm_analysed(brp, bci, vcol, masks, B, mb=mb, kb=mb, n=K, ldb=K, C=Ca, ldc=K)
    torch.cuda.synchronize()
    brp_h = brp.cpu().numpy()
    seg = _segmented_block_rows(brp_h)
    if kind == "reddit" and reorder:
        assert seg, "the RCM-reordered reddit stand-in must exercise the segmented rows"
    what = f"analysed bs32 {kind}{' RCM' if reorder else ''} (nnzb {nnzb})"
    rows = _sample_rows(brp_h, bs, n, 21 + 2 * reorder + (kind == "products"), seg)
    _check_oracle_rows(oracle, Ca, rp, ci, v, B, rows, TOL_F32, what)
    _check_oracle_all(oracle, Ca, rp, ci, v, B, TOL_F32, what)
    _within(Ca[:n], Cc, absd, 2 * TOL_F32, what + " vs CSR")
    assert not bool(Ca[n:].any()), "padding rows of C must be zero"
    assert torch.equal(Ca, Cd), what + ": differs from the drop-in column stream"


@pytest.mark.parametrize("reorder", [False, True])
def test_analysed_bs16_f16_full_size(oracle, device, reorder):
    """Config 5's bs 16 fp16 product (K = 512) on the analysed entry at full
    size, on the products stand-in and after RCM (14.3 M blocks): sampled rows
    against the f64 oracle of the same fp16 values, every row against the CSR
    kernel on the fp16-rounded values, and C bit-identical to the drop-in
    column stream."""
    ops = _ops()
    rp, ci, n = _graph("products", reorder)
    K, bs = 512, 16
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float16).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B16 = (torch.rand((mb * bs, K), device=device) * 2 - 1).half()
    Bf = B16[:n].float().contiguous()
    Cc = ops.gespmm_csrmm(drp, dci, dv, Bf)
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), Bf.abs())
    del Bf
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    del dci, dv
    bval16 = bval.half()
    del bval
    nnzb = int(bci.numel())
    Cd = torch.empty((mb * bs, K), device=device)
    ops.bsrmm_f16(brp, bci, bval16, B16, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cd, ldc=K)
    masks, vcol = ops.bsr16_analysis(bval16, nnzb=nnzb)
    del bval16
    Ca = torch.empty((mb * bs, K), device=device)
    ops.bsrmm_analysed_f16(brp, bci, vcol, masks, B16, mb=mb, kb=mb, n=K, ldb=K, C=Ca, ldc=K)
    torch.cuda.synchronize()
    what = f"analysed bs16 fp16 products{' RCM' if reorder else ''} (nnzb {nnzb})"
    rows = _sample_rows(brp.cpu().numpy(), bs, n, 31 + reorder)
    _check_oracle_rows(oracle, Ca, rp, ci, v, B16, rows, TOL_F16_ACC, what)
    _check_oracle_all(oracle, Ca, rp, ci, v, B16, TOL_F16_ACC, what)
    _within(Ca[:n], Cc, absd, 2 * TOL_F16_ACC, what + " vs CSR")
    assert torch.equal(Ca, Cd), what + ": differs from the drop-in column stream"


def test_nonfinite_contract_full_size(device):
    """The two non-finite contracts of Path B (include/spmm_hip.h,
    spmm_set_bsr_options) at full size on the reddit stand-in, bs 32: three B
    rows set to NaN. Expected NaN rows come from the block pattern on the host:
      * default (column-granular): every row of block row I iff a stored block
        (I, J) has a value other than +-0 in the column holding the NaN row;
      * SPMM_BSR_DENSE_BLOCK_PRODUCT (cusparseSbsrmm's dense blocks): every row
        of block row I iff a block (I, J) is stored at all.
    Everything else is finite and equals the CSR kernel on B with those rows
    zeroed, within the fp32 bar."""
    from spmm_hip import prep
    from spmm_hip._lib import BSR_DENSE_BLOCK_PRODUCT
    ops = _ops()
    rp, ci, n = _graph("reddit", False)
    K, bs = 128, 32
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    mb = (n + bs - 1) // bs
    # NaN rows: a hub column, a mid-popularity one and one past n's last block
    deg = np.bincount(ci, minlength=n)
    order = np.argsort(-deg, kind="stable")
    nan_rows = np.array(sorted({int(order[0]), int(order[n // 50]), n - 1}), dtype=np.int64)
    drp, dci, dv = _dev(rp, ci, v)
    B = torch.rand((mb * bs, K), device=device) * 2 - 1
    B0 = B.clone()
    B0[torch.from_numpy(nan_rows).to(device)] = 0.0
    B[torch.from_numpy(nan_rows).to(device)] = float("nan")
    Cc = ops.gespmm_csrmm(drp, dci, dv, B0[:n].contiguous())
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B0[:n].abs().contiguous())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    brp_h, bci_h = brp.cpu().numpy(), bci.cpu().numpy()
    # column-granular: (block row, column) pairs holding a nonzero, from the CSR pattern
    row_of = np.repeat(np.arange(n), np.diff(rp))
    hit_col = np.zeros(mb, bool)
    for r in nan_rows:
        hit_col[np.unique(row_of[ci == r] // bs)] = True
    blk_row_of = np.repeat(np.arange(mb), np.diff(brp_h))
    hit_dense = np.zeros(mb, bool)
    for r in nan_rows:
        hit_dense[np.unique(blk_row_of[bci_h == r // bs])] = True
    assert hit_dense.sum() > hit_col.sum() > 0, "the case must separate the two contracts"
    for flags, hit in ((0, hit_col), (BSR_DENSE_BLOCK_PRODUCT, hit_dense)):
        h = ops.Handle()
        h.set_bsr_options(flags)
        C = torch.empty((mb * bs, K), device=device)
        ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K, handle=h)
        torch.cuda.synchronize()
        nanrow = torch.isnan(C).view(mb, bs * K)
        want = torch.from_numpy(hit).to(device)
        got_any, got_all = nanrow.any(dim=1), nanrow.all(dim=1)
        assert torch.equal(got_any, want) and torch.equal(got_all, want), (
            f"flags {flags}: NaN block rows {int(got_any.sum())} (whole: {int(got_all.sum())}), "
            f"expected {int(want.sum())}")
        keep = ~want.repeat_interleave(bs)[:n]
        _within(C[:n][keep], Cc[keep], absd[keep], 2 * TOL_F32, f"flags {flags}: finite rows vs CSR")
        h.close()


@pytest.mark.parametrize("W,reorder", [(4, False), (8, False), (4, True)])
def test_grouped_bs16_f16_full_size(oracle, device, W, reorder):
    """Config 5's product on the grouped stream at full size (products stand-in,
    K = 512; after RCM too: 14.3 M blocks): sampled rows against the f64 oracle
    of the same fp16 values and every row against the CSR kernel on the
    fp16-rounded values."""
    ops = _ops()
    rp, ci, n = _graph("products", reorder)
    K, bs = 512, 16
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float16).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B16 = (torch.rand((mb * bs, K), device=device) * 2 - 1).half()
    Bf = B16[:n].float().contiguous()
    Cc = ops.gespmm_csrmm(drp, dci, dv, Bf)
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), Bf.abs())
    del Bf
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    del dci, dv
    bval16 = bval.half()
    del bval
    grp = ops.GroupedBsr16(brp, bci, bval16, mb=mb, group_rows=W)
    del bval16
    Cg = torch.empty((mb * bs, K), device=device)
    grp.mm(B16, kb=mb, n=K, ldb=K, C=Cg, ldc=K)
    torch.cuda.synchronize()
    what = f"grouped W={W} bs16 fp16 products{' RCM' if reorder else ''}"
    rows = _sample_rows(brp.cpu().numpy(), bs, n, 41 + W + reorder)
    _check_oracle_rows(oracle, Cg, rp, ci, v, B16, rows, TOL_F16_ACC, what)
    _check_oracle_all(oracle, Cg, rp, ci, v, B16, TOL_F16_ACC, what)
    _within(Cg[:n], Cc, absd, 2 * TOL_F16_ACC, what + " vs CSR")
    assert not bool(Cg[n:].any()), "padding rows of C must be zero"
    grp.close()


def test_grouped_bs16_nonfinite_contract_full_size(device):
    """The grouped stream's non-finite contract at full size: the products
    stand-in at K = 512, W = 4, three B rows set to NaN (a hub column, a
    mid-popularity one and n - 1). Since round 5 it is the drop-in stream's
    column-granular contract: the NaN block rows must be exactly those holding
    a value in a NaN row's column (predicted from the CSR pattern), a strict
    subset of their groups (round 4's GROUPED contract). Every other element
    equals the run on B with those rows zeroed, bit for bit."""
    ops = _ops()
    rp, ci, n = _graph("products", False)
    K, bs, W = 512, 16, 4
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float16).astype(np.float32)
    mb = (n + bs - 1) // bs
    deg = np.bincount(ci, minlength=n)
    order = np.argsort(-deg, kind="stable")
    nan_rows = np.array(sorted({int(order[0]), int(order[n // 50]), n - 1}), dtype=np.int64)
    row_of = np.repeat(np.arange(n), np.diff(rp))
    hit_col = np.zeros(mb, bool)  # column-granular
    for r in nan_rows:  # a value that rounds to fp16 zero leaves its column empty
        hit_col[np.unique(row_of[(ci == r) & (v != 0)] // bs)] = True
    ngrp = -(-mb // W)
    hit_grp = np.repeat(np.pad(hit_col, (0, ngrp * W - mb)).reshape(ngrp, W).any(axis=1), W)[:mb]
    assert hit_grp.sum() > hit_col.sum() > 0, "the case must separate the two contracts"
    drp, dci, dv = _dev(rp, ci, v)
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    del drp, dci, dv
    bval16 = bval.half()
    del bval
    grp = ops.GroupedBsr16(brp, bci, bval16, mb=mb, group_rows=W)
    del bval16
    B = (torch.rand((mb * bs, K), device=device) * 2 - 1).half()
    idx = torch.from_numpy(nan_rows).to(device)
    B0 = B.clone()
    B0[idx] = 0
    B[idx] = float("nan")
    C = torch.empty((mb * bs, K), device=device)
    grp.mm(B, kb=mb, n=K, ldb=K, C=C, ldc=K)
    C0 = torch.empty((mb * bs, K), device=device)
    grp.mm(B0, kb=mb, n=K, ldb=K, C=C0, ldc=K)
    torch.cuda.synchronize()
    grp.close()
    nanrow = torch.isnan(C).view(mb, bs * K)
    want = torch.from_numpy(hit_col).to(device)
    assert torch.equal(nanrow.any(dim=1), want) and torch.equal(nanrow.all(dim=1), want), (
        f"NaN block rows {int(nanrow.any(dim=1).sum())} (whole: {int(nanrow.all(dim=1).sum())}), "
        f"expected {int(want.sum())}")
    keep = ~want.repeat_interleave(bs)
    assert torch.equal(C[keep], C0[keep]), "finite rows differ from the zeroed-B run"


@pytest.mark.parametrize("kind,reorder,W", [("reddit", False, 2), ("reddit", True, 2),
                                            ("products", False, 2), ("products", False, 4)])
def test_grouped_bs32_full_size(oracle, device, kind, reorder, W):
    """Config 3's bs 32 fp32 product on the grouped bs 32 stream at full size
    (reddit, RCM reddit, products at 2 and 4 block rows per group): sampled rows
    against the f64 oracle, every row against the CSR kernel, and C bit-identical
    to the drop-in column stream wherever that stream runs whole block rows (the
    segmented outlier rows of RCM reddit sum their partials in another order:
    there the bar is the oracle's)."""
    ops = _ops()
    rp, ci, n = _graph(kind, reorder)
    K, bs = 128, 32
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=device) * 2 - 1
    Cc = ops.gespmm_csrmm(drp, dci, dv, B[:n].contiguous())
    absd = ops.gespmm_csrmm(drp, dci, dv.abs(), B[:n].abs().contiguous())
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    del dci, dv
    Cd = torch.empty((mb * bs, K), device=device)
    ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=Cd, ldc=K)
    grp = ops.GroupedBsr32(brp, bci, bval, mb=mb, group_rows=W)
    del bval
    Cg = torch.empty((mb * bs, K), device=device)
    grp.mm(B, kb=mb, n=K, ldb=K, C=Cg, ldc=K)
    torch.cuda.synchronize()
    brp_h = brp.cpu().numpy()
    seg = _segmented_block_rows(brp_h)
    what = f"grouped W={W} bs32 {kind}{' RCM' if reorder else ''}"
    rows = _sample_rows(brp_h, bs, n, 61 + W + 2 * reorder + (kind == "products"), seg)
    _check_oracle_rows(oracle, Cg, rp, ci, v, B, rows, TOL_F32, what)
    _check_oracle_all(oracle, Cg, rp, ci, v, B, TOL_F32, what)
    _within(Cg[:n], Cc, absd, 2 * TOL_F32, what + " vs CSR")
    assert not bool(Cg[n:].any()), "padding rows of C must be zero"
    # every segmented block row (seg above holds the shortest and the longest)
    nbr = np.diff(brp_h)
    same = torch.ones(mb, dtype=torch.bool)
    if seg:
        same[torch.from_numpy(nbr >= nbr[seg[0]])] = False
    eq = (Cg.view(mb, bs, K) == Cd.view(mb, bs, K)).all(dim=2).all(dim=1).cpu()
    bad = same & ~eq
    assert not bool(bad.any()), (f"{what}: {int(bad.sum())} whole block rows differ from the "
                                 f"drop-in column stream")
    grp.close()
