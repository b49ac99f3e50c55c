"""Path B at BASELINE's full sizes, through
size-independent properties: the BSR, hybrid and CSR kernels are three
independent implementations of the same product, so at full scale each BSR
result must agree with the CSR kernel's within the fp32 bar, with the
magnitude bound |A|.|B| itself computed on the device (the CSR kernel on
|val|, |B|). The small-size tests pin each kernel to the oracle; these check
that nothing breaks at 10^8 nonzeros (index widths, grid sizes, tails)."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import TOL_F16_ACC, TOL_F32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ops():
    from spmm_hip import ops
    return ops


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _within(got, ref, absd, tol, what):
    err = (got - ref).abs()
    bound = tol * absd + 1e-30
    bad = int((err > bound).sum())
    assert bad == 0, f"{what}: {bad} elements outside {tol} x |A||B| (max err {float(err.max())})"


def test_reddit_scale_bsr32_and_hybrid_vs_csr(device):
    """Config 3 (reddit stand-in, 115 M nnz, bs = 32, K = 128): device csr2bsr
    -> LDS MFMA kernel, and divide -> hybrid, both against the CSR kernel."""
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
        _within(Ch[:n], Cc, absd, 2 * TOL_F32, f"reddit hybrid (flags {flags}) vs CSR")
        h.close()


def test_products_scale_bsr16_f16_vs_csr(device):
    """Config 5 (products stand-in, bs = 16, fp16 A and B, K = 512): the
    fp16 MFMA kernel against the CSR kernel run on the same fp16-rounded
    values in fp32 (both accumulate in fp32)."""
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
    _within(Cb[:n], Cc, absd, 2 * TOL_F16_ACC, "products bs16 fp16 BSR vs CSR")


@pytest.mark.parametrize("bs", [32, 16])
def test_reordered_reddit_scale_bsr_vs_csr(device, bs):
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
        _within(Ch[:n], Cc, absd, 2 * TOL_F32, "RCM-reordered reddit hybrid vs CSR")
