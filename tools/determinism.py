"""Run-to-run determinism of the shipped kernels at BASELINE sizes: every
default path is written to be deterministic (no float atomics; fixed
reduction orders), so repeated runs on the same inputs must agree bit for
bit. A difference points at a copy/compute race like the one the CM4 kernel
had. GPU box only; diagnostic, not a test.

usage: python tools/determinism.py [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "spmm-denseblock_amd"))
from spmm_hip import ops, prep  # noqa: E402


def check(tag, run, reps):
    first = run().clone()
    torch.cuda.synchronize()
    diffs = []
    for _ in range(reps):
        out = run()
        torch.cuda.synchronize()
        diffs.append(int((out != first).sum()))
    print(f"{tag}: differing elements per rerun {diffs}", flush=True)
    return sum(diffs)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda:0")
    bad = 0
    # products stand-in (community order): CSR K=128, bs 32 column stream and its
    # analysed form, bs 16 fp16 K=512 (drop-in, analysed, grouped), hybrid fused
    # (plain and split-bf16), device csr2bsr
    n = 2449029
    rp, ci = prep.community_csr(n, 27.0, 32, 512, 0.97, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = [torch.from_numpy(a).to(dev) for a in (rp, ci, v)]
    torch.manual_seed(0)
    for bs, K in ((32, 128), (16, 512)):
        mb = (n + bs - 1) // bs
        B = torch.rand((mb * bs, K), device=dev) * 2 - 1
        if bs == 32:
            Bn = B[:n].contiguous()
            bad += check("csr K=128", lambda: ops.gespmm_csrmm(drp, dci, dv, Bn), reps)
            tag = ops.csr_hot_analysis(dci, n=K, k=n)
            bad += check("csr hot-column tags", lambda: ops.csr_hot_analysis(dci, n=K, k=n), 2)
            Ch = torch.empty((n, K), device=dev)

            def run_hot():
                ops.csrmm_hot(drp, tag, dv, Bn, n=K, k=n, ldb=K, C=Ch, ldc=K)
                return Ch
            bad += check("csr K=128 (hot-column hints)", run_hot, reps)
            ref = ops.gespmm_csrmm(drp, dci, dv, Bn)
            bad += int((run_hot() != ref).sum())
            # grid independence: other grids, the _ex entry, row shards
            from spmm_hip import dist as sdist
            for wpc in (4, 16, 32):
                hx = ops.Handle()
                hx.set_csr_waves_per_cu(wpc)
                ops.csrmm(drp, dci, dv, Bn, n=K, k=n, ldb=K, C=Ch, ldc=K, handle=hx)
                torch.cuda.synchronize()
                d = int((Ch != ref).sum())
                print(f"csr K=128 _ex entry, {wpc} waves/CU vs the drop-in: {d} differing",
                      flush=True)
                bad += d
                hx.close()
            for world in (2, 8):
                Ch.fill_(float("nan"))
                for r in range(world):
                    sh = sdist.make_shard(rp, ci, v, r, world)
                    srp, sci, sv = [torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                                    for a in (sh.rowptr, sh.colind, sh.val)]
                    ops.csrmm(srp, sci, sv, Bn, m=sh.rows, n=K, k=n, ldb=K,
                              C=Ch[sh.row0:sh.row1], ldc=K)
                torch.cuda.synchronize()
                d = int((Ch != ref).sum())
                print(f"csr K=128 {world} row shards vs the whole matrix: {d} differing",
                      flush=True)
                bad += d
            del Bn, tag, Ch, ref
        bad += check(f"csr2bsr bs={bs} (values)",
                     lambda: ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)[2], 2)
        brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
        C = torch.empty((mb * bs, K), device=dev)
        if bs == 32:
            def run():
                ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K)
                return C
            bad += check("bsr32 fp32 K=128 (column stream, CS2)", run, reps)
            masks, vcol = ops.bsr32_analysis(bval, nnzb=bci.numel())

            def run_an():
                ops.bsrmm_analysed(brp, bci, vcol, masks, B, mb=mb, kb=mb, n=K, ldb=K, C=C, ldc=K)
                return C
            bad += check("bsr32 fp32 K=128 (analysed column stream)", run_an, reps)
            del masks, vcol
            g32 = ops.GroupedBsr32(brp, bci, bval, mb=mb, group_rows=2)

            def run_g32():
                g32.mm(B, kb=mb, n=K, ldb=K, C=C, ldc=K)
                return C
            bad += check("bsr32 fp32 K=128 (grouped stream, 2 block rows)", run_g32, reps)
            g32.close()
            del g32
        else:
            bv16, B16 = bval.half(), B.half()
            del bval, B

            def run():
                ops.bsrmm_f16(brp, bci, bv16, B16, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K)
                return C
            bad += check("bsr16 fp16 K=512 (column stream, CS16)", run, reps)
            masks16, vcol16 = ops.bsr16_analysis(bv16, nnzb=bci.numel())

            def run_an16():
                ops.bsrmm_analysed_f16(brp, bci, vcol16, masks16, B16, mb=mb, kb=mb, n=K, ldb=K,
                                       C=C, ldc=K)
                return C
            bad += check("bsr16 fp16 K=512 (analysed column stream)", run_an16, reps)
            del masks16, vcol16
            g = ops.GroupedBsr16(brp, bci, bv16, mb=mb, group_rows=4)

            def run_grp():
                g.mm(B16, kb=mb, n=K, ldb=K, C=C, ldc=K)
                return C
            bad += check("bsr16 fp16 K=512 (grouped stream, 4 block rows)", run_grp, reps)
            g.close()
            del g
            del bv16, B16
        del brp, bci, C
        torch.cuda.empty_cache()
    from spmm_hip._lib import HYBRID_SPLIT_BF16
    K, bs = 128, 32
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=dev) * 2 - 1
    parts = prep.divide(n, rp, ci, v, bs, prep.hybrid_plan(rp, ci, bs, K)["density"])
    d = [torch.from_numpy(a).to(dev) for a in parts]
    C = torch.empty((mb * bs, K), device=dev)
    for flags in (0, HYBRID_SPLIT_BF16):
        h = ops.Handle()
        h.set_hybrid_options(flags)

        def run():
            ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), B, m=n, n=K, k=n, bs=bs, ldb=K, C=C,
                             ldc=K, handle=h)
            return C
        bad += check(f"hybrid fused flags={flags}", run, reps)
        h.close()
    del d, C, B
    torch.cuda.empty_cache()
    # community-ordered reddit stand-in, bs 8 / 2: the grouped small-bs MFMA stream (merge in
    # LDS, longest-first groups; reddit_bsr8 / reddit_bsr2)
    n = 232965
    rp, ci = prep.community_csr(n, 670.0, 512, 2048, 0.99, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = [torch.from_numpy(a).to(dev) for a in (rp, ci, v)]
    for bs2 in (8, 2):
        mb2 = (n + bs2 - 1) // bs2
        B2 = torch.rand((mb2 * bs2, K), device=dev) * 2 - 1
        C2 = torch.empty((mb2 * bs2, K), device=dev)
        brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs2)

        def run():
            ops.bsrmm(brp, bci, bval, B2, mb=mb2, kb=mb2, n=K, bs=bs2, ldb=K, C=C2, ldc=K)
            return C2
        bad += check(f"reddit bsr{bs2} (grouped small-bs stream)", run, reps)
        del brp, bci, bval, B2, C2
        torch.cuda.empty_cache()
    del drp, dci, dv
    # RCM-reordered reddit stand-in, bs 32: the longest-first order with
    # segments of the outlier rows (partial tiles + fix-up) and the fused
    # hybrid on the same matrix (longest-first order)
    rp, ci = prep.permute_csr(rp, ci, np.random.default_rng(9).permutation(n).astype(np.int32))
    rp, ci = prep.permute_csr(rp, ci, prep.reorder(rp, ci, "rcm"))
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = [torch.from_numpy(a).to(dev) for a in (rp, ci, v)]
    mb = (n + bs - 1) // bs
    B = torch.rand((mb * bs, K), device=dev) * 2 - 1
    brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs)
    C = torch.empty((mb * bs, K), device=dev)

    def run():
        ops.bsrmm(brp, bci, bval, B, mb=mb, kb=mb, n=K, bs=bs, ldb=K, C=C, ldc=K)
        return C
    bad += check("RCM reddit bsr32 (segments)", run, reps)
    parts = prep.divide(n, rp, ci, v, bs, prep.hybrid_plan(rp, ci, bs, K)["density"])
    d = [torch.from_numpy(a).to(dev) for a in parts]

    def run():
        ops.hybrid_csrmm(tuple(d[0:3]), tuple(d[3:6]), B, m=n, n=K, k=n, bs=bs, ldb=K, C=C, ldc=K)
        return C
    bad += check("RCM reddit hybrid (fused, longest first)", run, reps)
    del d, brp, bci, bval
    # bs 8 (lane-group VALU kernel) and bs 64 (the bs 32 column stream on sub-blocks)
    for bs2 in (8, 64):
        mb2 = (n + bs2 - 1) // bs2
        B2 = torch.rand((mb2 * bs2, K), device=dev) * 2 - 1
        C2 = torch.empty((mb2 * bs2, K), device=dev)
        brp, bci, bval = ops.csr2bsr(drp, dci, dv, m=n, n=n, bs=bs2)

        def run():
            ops.bsrmm(brp, bci, bval, B2, mb=mb2, kb=mb2, n=K, bs=bs2, ldb=K, C=C2, ldc=K)
            return C2
        bad += check(f"RCM reddit bsr{bs2}", run, reps)
        del brp, bci, bval, B2, C2
        torch.cuda.empty_cache()
    # the bs 32 panel stream (dense blocks, the reference sweep's test_bsrmm matrices): reruns,
    # both C layouts, and its bits against the analysed column stream's
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    mbp, per_row, K = 2048, 60, 128
    bci = torch.sort(torch.rand((mbp, mbp), device=dev, generator=g).argsort(dim=1)[:, :per_row],
                     dim=1)[0].to(torch.int32).reshape(-1).contiguous()
    brp = torch.arange(0, mbp * per_row + 1, per_row, dtype=torch.int32, device=dev)
    bval = torch.rand(bci.numel() * 1024, device=dev, generator=g) * 2 - 1
    B = torch.rand((mbp * 32, K), device=dev, generator=g) * 2 - 1
    masks, vcol = ops.bsr32_analysis(bval, nnzb=bci.numel())
    for oc, tag in ((ops.ORDER_ROW, "row-major C"), (ops.ORDER_COL, "column-major C")):
        C = torch.empty(mbp * 32 * K, device=dev)
        ld = K if oc == ops.ORDER_ROW else mbp * 32

        def run_p(C=C, oc=oc, ld=ld):
            ops.bsrmm(brp, bci, bval, B, mb=mbp, kb=mbp, n=K, bs=32, ldb=K, C=C, ldc=ld, order_c=oc)
            return C
        bad += check(f"bsr32 fp32 K=128 dense blocks (panel stream, {tag})", run_p, reps)
        C2 = torch.empty_like(C)
        ops.bsrmm_analysed(brp, bci, vcol, masks, B, mb=mbp, kb=mbp, n=K, ldb=K, C=C2, ldc=ld,
                           order_c=oc)
        torch.cuda.synchronize()
        d = int((run_p() != C2).sum())
        print(f"bsr32 dense blocks ({tag}): panel stream vs the analysed column stream: {d} differing",
              flush=True)
        bad += d
    print(f"total differing elements: {bad}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
