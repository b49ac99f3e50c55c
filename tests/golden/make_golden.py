"""Generates the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference and `make -C oracle ref`):
    python tests/golden/make_golden.py

Two kinds of fixtures:
  kats.json    The reference's own known-answer programs (inputs copied as
               data from csrmm.cu, bsrmm.cu, block_cublas.cu, try_cublas.cu,
               spmm.cc). Those programs only print their result; the expected
               outputs here are computed with numpy (float64) from the inputs
               and the documented layout semantics of the cuSPARSE/cuBLAS call
               each program makes, and are cross-checked against the values
               listed in SURVEY.md §4.
  ref_*.npz    Outputs of the reference's OWN host code (load_data.cc RNG and
               generators, utility.cc calculateNnzb, divide.cu divide_matrix)
               compiled from /root/reference into oracle/_ref/libref.so by
               oracle/Makefile. These pin the RNG stream and the csr2bsr index
               arrays bit-exactly; the GPU box (no reference tree) uses them.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIBREF = os.path.join(ROOT, "oracle", "_ref", "libref.so")


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def kats() -> dict:
    out = {}
    # csrmm.cu:47-99 (COO -> coo2csr), y col-major 4x2, cusparseScsrmm
    # (csrmm.cu:183-185: m=n=4, K=2, ldb=ldc=4), C col-major.
    rows = [0, 0, 0, 1, 2, 2, 2, 3, 3]
    cols = [0, 2, 3, 1, 0, 2, 3, 1, 3]
    vals = [1, 2, 3, 4, 5, 6, 7, 8, 9]
    A = np.zeros((4, 4))
    A[rows, cols] = vals
    y = np.array([10, 20, 30, 40, 50, 60, 70, 80], float).reshape(2, 4).T  # col-major 4x2
    z = A @ y
    rp = np.searchsorted(rows, np.arange(5)).tolist()
    out["csrmm_cu"] = dict(src="csrmm.cu:47-99,148-149,183-185", m=4, k=4, n=2, coo_row=rows,
                           rowptr=rp,
                           colind=cols, val=vals, B_colmajor=[10, 20, 30, 40, 50, 60, 70, 80],
                           ldb=4, ldc=4, C_colmajor=z.T.reshape(-1).tolist(),
                           survey=[190, 80, 510, 520, 430, 240, 1230, 1200])
    # bsrmm.cu:50-61 (mb=2, kb=3, bs=2, n=2, DIRECTION_ROW), y 6x2 col-major,
    # cusparseSbsrmm (bsrmm.cu:141-144: ldb = k = 6, ldc = m = 4).
    brp, bci = [0, 2, 4], [0, 2, 1, 2]
    bval = [0, 4, 2, 7, 1, 8, 2, 0, 9, 0, 0, 2, 0, 6, 7, 0]
    A = np.zeros((4, 6))
    for br in range(2):
        for kk in range(brp[br], brp[br + 1]):
            blk = np.array(bval[4 * kk:4 * kk + 4], float).reshape(2, 2)  # row-major block
            A[2 * br:2 * br + 2, 2 * bci[kk]:2 * bci[kk] + 2] = blk
    y = np.arange(1, 13, dtype=float).reshape(2, 6).T
    z = A @ y
    out["bsrmm_cu"] = dict(src="bsrmm.cu:50-61,141-144", mb=2, kb=3, n=2, bs=2, dir=0,
                           rowptr=brp, colind=bci, val=bval, B_colmajor=list(range(1, 13)),
                           ldb=6, ldc=4, C_colmajor=z.T.reshape(-1).tolist(),
                           survey=[61, 26, 63, 43, 139, 92, 153, 97])
    # block_cublas.cu:49-56,87-90,123-136: per block cublasSgemm(N, T, bs, K, bs)
    # with A block col-major (lda = bs), Y row-major (ldb = K), C col-major
    # (ldc = m), beta = 1 onto zeroed C  ==  bsrmm dir=COLUMN, B row-major.
    brp, bci = [0, 2, 3], [0, 1, 1]
    bval = [0, 3, 1, 2, 4, 2, 0, 0, 0, 5, 0, 8]
    A = np.zeros((4, 4))
    for br in range(2):
        for kk in range(brp[br], brp[br + 1]):
            blk = np.array(bval[4 * kk:4 * kk + 4], float).reshape(2, 2).T  # col-major block
            A[2 * br:2 * br + 2, 2 * bci[kk]:2 * bci[kk] + 2] = blk
    Y = np.array([6, 0, 0, 0, 7, 5, 4, 3, 0, 0, 0, 7], float).reshape(4, 3)
    z = A @ Y
    out["block_cublas_cu"] = dict(src="block_cublas.cu:49-56,123-136", mb=2, kb=2, n=3, bs=2,
                                  dir=1, rowptr=brp, colind=bci, val=bval,
                                  B_rowmajor=Y.reshape(-1).tolist(), ldb=3, ldc=4, beta=1.0,
                                  C_colmajor=z.T.reshape(-1).tolist(),
                                  survey=[16, 26, 0, 20, 19, 20, 0, 15, 5, 10, 0, 56])
    # try_cublas.cu:54-79: cublasSgemm(N, N, m=2, n=4, k=3), A col-major 2x3,
    # B col-major 3x4 -> as a fully dense CSR A times col-major B.
    Ad = np.array([1, 4, 2, 5, 3, 6], float).reshape(3, 2).T
    Bd = np.array([1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0], float).reshape(4, 3).T
    z = Ad @ Bd
    out["try_cublas_cu"] = dict(src="try_cublas.cu:54-79", m=2, k=3, n=4,
                                rowptr=[0, 3, 6], colind=[0, 1, 2, 0, 1, 2],
                                val=Ad.reshape(-1).tolist(),
                                B_colmajor=[1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0], ldb=3, ldc=2,
                                C_colmajor=z.T.reshape(-1).tolist(),
                                survey=[4, 10, 2, 5, 4, 10, 2, 5])
    # spmm.cc:45-52 test_small_csr_spmm: pattern-only CSR x row-major dense.
    ip, ix = [0, 1, 3], [1, 0, 2]
    D = np.array([[3, 9, 2], [4, 6, 7], [5, 8, 1]], float)
    Ap = np.zeros((2, 3))
    for r in range(2):
        Ap[r, ix[ip[r]:ip[r + 1]]] = 1
    out["spmm_cc_small"] = dict(src="spmm.cc:45-52", m=2, k=3, n=3, indptr=ip, indices=ix,
                                dense=D.reshape(-1).tolist(), out=(Ap @ D).reshape(-1).tolist(),
                                survey=[4, 6, 7, 8, 17, 3])
    for name, d in out.items():
        key = "C_colmajor" if "C_colmajor" in d else "out"
        assert np.array_equal(np.array(d[key]), np.array(d["survey"], float)), name
    return out


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_fixtures():
    L = ctypes.CDLL(LIBREF)
    L.ref_seed.argtypes = [ctypes.c_uint64]
    L.ref_random_dense.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_void_p]
    L.ref_random_csr.restype = ctypes.c_int64
    L.ref_random_csr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int64]
    L.ref_random_bsr.restype = ctypes.c_int64
    L.ref_random_bsr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    L.ref_calculate_nnzb.restype = ctypes.c_int64
    L.ref_calculate_nnzb.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int]
    L.ref_divide_matrix.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_float, ctypes.c_void_p]
    L.ref_divide_fetch.argtypes = [ctypes.c_void_p] * 5

    def rcsr(m, n, p, lo=-1.0, hi=1.0):
        cap = int(m * n * p * 1.5) + 1024
        rp = np.zeros(m + 1, np.int32)
        ci = np.zeros(cap, np.int32)
        v = np.zeros(cap, np.float32)
        nnz = L.ref_random_csr(m, n, p, lo, hi, _p(rp), _p(ci), _p(v), cap)
        assert nnz >= 0
        return rp, ci[:nnz].copy(), v[:nnz].copy()

    fx = {}
    # RNG stream (load_data.cc:12,29-40) from a fresh generator.
    L.ref_seed(1234)
    d = np.zeros(4096, np.float32)
    L.ref_random_dense(64, 64, -1.0, 1.0, _p(d))
    fx["dense_64x64"] = d
    # randomCSRMatrix at the sizes the parity tests use (fresh generator each).
    for (m, n, p) in [(64, 80, 0.1), (300, 257, 0.03), (1000, 1200, 0.01)]:
        L.ref_seed(1234)
        rp, ci, v = rcsr(m, n, p)
        fx[f"csr_{m}_{n}_{p}_rowptr"] = rp
        fx[f"csr_{m}_{n}_{p}_colind"] = ci
        fx[f"csr_{m}_{n}_{p}_val"] = v
    # randomBSRMatrix (load_data.cc:81-113).
    L.ref_seed(1234)
    mb, nb, bs, p = 12, 10, 4, 0.2
    cap = mb * nb
    rp = np.zeros(mb + 1, np.int32)
    ci = np.zeros(cap, np.int32)
    v = np.zeros(cap * bs * bs, np.float32)
    nnzb = L.ref_random_bsr(mb, nb, bs, p, -1.0, 1.0, _p(rp), _p(ci), _p(v), cap)
    fx["bsr_12_10_4_rowptr"], fx["bsr_12_10_4_colind"] = rp, ci[:nnzb].copy()
    fx["bsr_12_10_4_val"] = v[:nnzb * bs * bs].copy()
    # divide_matrix at density 1e-9 == csr2bsr (DIRECTION_ROW, unit values) and
    # calculateNnzb, on the (300, 257) pattern (square view: n = 300 rows,
    # columns < 257) and a banded pattern, for several block sizes.
    rp300, ci300 = fx["csr_300_257_0.03_rowptr"], fx["csr_300_257_0.03_colind"]
    band_rp = [0]
    band_ci = []
    for r in range(200):
        cs = sorted({c for c in range(max(0, r - 5), min(200, r + 6)) if (r * 7 + c) % 3})
        band_ci += cs
        band_rp.append(len(band_ci))
    graphs = {"rand300": (rp300, ci300, 300),
              "band200": (np.array(band_rp, np.int32), np.array(band_ci, np.int32), 200)}
    for gname, (grp, gci, n) in graphs.items():
        fx[f"{gname}_rowptr"], fx[f"{gname}_colind"] = grp, gci
        for bs in (2, 4, 16, 32):
            sizes = np.zeros(5, np.int64)
            for density, tag in ((1e-9, "all"), (0.25, "d25")):
                L.ref_divide_matrix(n, _p(grp), _p(gci), bs, density, _p(sizes))
                arrs = [np.zeros(int(s), t) for s, t in
                        zip(sizes, [np.int32, np.int32, np.int32, np.int32, np.float32])]
                L.ref_divide_fetch(*[_p(a) if a.size else ctypes.c_void_p(0) for a in arrs])
                for nm, a in zip(["csr_rp", "csr_ci", "bsr_rp", "bsr_ci", "bsr_val"], arrs):
                    fx[f"{gname}_bs{bs}_{tag}_{nm}"] = a
            fx[f"{gname}_bs{bs}_nnzb"] = np.array(
                [L.ref_calculate_nnzb(n, _p(grp), _p(gci), bs)], np.int64)
    return fx


def reorder_graphs(fx_host: dict) -> dict:
    """Inputs of the reorder fixtures: the two divide graphs, a power-law
    graph with many equal degrees, isolated nodes and several components,
    and a scrambled community graph (what a reorder should un-scramble)."""
    g = {"rand300": (fx_host["rand300_rowptr"], fx_host["rand300_colind"]),
         "band200": (fx_host["band200_rowptr"], fx_host["band200_colind"])}
    rng = np.random.default_rng(77)
    n = 2000
    deg = np.minimum((rng.zipf(2.1, n) - 1) * 2, 400)
    deg[rng.choice(n, 50, replace=False)] = 0  # isolated rows
    rows = [np.sort(rng.choice(n, d, replace=False)) for d in deg]
    g["pl2000"] = (np.concatenate([[0], np.cumsum(deg)]).astype(np.int32),
                   np.concatenate(rows).astype(np.int32))
    n, rows = 1500, []
    comm = np.repeat(np.arange(15), 100)
    for r in range(n):
        inside = rng.choice(np.flatnonzero(comm == comm[r]), 12, replace=False)
        outside = rng.choice(n, 2, replace=False)
        rows.append(np.union1d(inside, outside))
    perm = rng.permutation(n)  # scramble: old -> new
    srows = [None] * n
    for r in range(n):
        srows[perm[r]] = np.sort(perm[rows[r]])
    g["comm1500"] = (np.concatenate([[0], np.cumsum([len(x) for x in srows])]).astype(np.int32),
                     np.concatenate(srows).astype(np.int32))
    return g


def reorder_fixtures(fx_host: dict, tmpdir: str) -> dict:
    """The reference's own reorder front-end (reorder_strategy.cc,
    utility.cc getHeatmap, rabbit_reorder.cc loadPermutation, reorder_graph.cc
    analyzeBlockSparseMetrics) on reorder_graphs()."""
    L = ctypes.CDLL(LIBREF)
    L.ref_reorder.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
    L.ref_heatmap.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p]
    L.ref_load_permutation.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    L.ref_block_metrics_text.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    fx = {}
    for name, (rp, ci) in reorder_graphs(fx_host).items():
        n, nnz = rp.size - 1, ci.size
        fx[f"{name}_rowptr"], fx[f"{name}_colind"] = rp, ci
        perm = np.random.default_rng(n).permutation(n).astype(np.int32)
        fx[f"{name}_perm"] = perm
        for kind, tag in ((0, "degree"), (1, "bfs"), (2, "rcm"), (3, "permute")):
            orp, oci = np.zeros(n + 1, np.int32), np.zeros(nnz, np.int32)
            assert L.ref_reorder(kind, n, _p(rp), _p(ci), _p(perm), _p(orp), _p(oci)) == 0
            fx[f"{name}_{tag}_rowptr"], fx[f"{name}_{tag}_colind"] = orp, oci
        for bs in (16, 64):
            nb = (n + bs - 1) // bs
            h = np.zeros(nb * nb, np.int32)
            L.ref_heatmap(n, _p(rp), _p(ci), bs, _p(h))
            fx[f"{name}_heatmap{bs}"] = h
        buf = ctypes.create_string_buffer(1 << 14)
        ln = L.ref_block_metrics_text(n, _p(rp), _p(ci), nnz, buf, len(buf))
        assert ln > 0
        fx[f"{name}_metrics_text"] = np.array(buf.value.decode())
        # loadPermutation on a file in the rabbit/Gorder format.
        f = os.path.join(tmpdir, f"{name}_perm.txt")
        with open(f, "w") as fh:
            fh.write("\n".join(str(x) for x in perm) + "\n")
        got = np.zeros(n, np.int32)
        L.ref_load_permutation(f.encode(), n, _p(got))
        assert np.array_equal(got, perm)
    return fx


def big_digest():
    """Config 1 (BASELINE configs[0]): randomCSRMatrix(16384, 16384, 2^-10)
    from a fresh generator, followed by randomDenseMatrix(16384, 32):
    digests only (the arrays would be MBs)."""
    L = ctypes.CDLL(LIBREF)
    L.ref_seed.argtypes = [ctypes.c_uint64]
    L.ref_random_csr.restype = ctypes.c_int64
    L.ref_random_csr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int64]
    L.ref_random_dense.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_void_p]
    L.ref_seed(1234)
    m = 16384
    cap = 400000
    rp = np.zeros(m + 1, np.int32)
    ci = np.zeros(cap, np.int32)
    v = np.zeros(cap, np.float32)
    nnz = L.ref_random_csr(m, m, 2.0 ** -10, -1.0, 1.0, _p(rp), _p(ci), _p(v), cap)
    ci, v = ci[:nnz], v[:nnz]
    B = np.zeros(m * 32, np.float32)
    L.ref_random_dense(m, 32, -1.0, 1.0, _p(B))
    return dict(m=m, n=m, p=2.0 ** -10, K=32, nnz=int(nnz), rowptr_sha256=sha(rp),
                colind_sha256=sha(ci), val_sha256=sha(v), B_sha256=sha(B),
                rowptr_head=rp[:9].tolist(), colind_head=ci[:8].tolist(),
                val_head=v[:4].tolist(), B_head=B[:4].tolist())


def main():
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    if not os.path.exists(LIBREF):
        sys.exit("oracle/_ref/libref.so missing: run `make -C oracle ref` first")
    host = ref_fixtures()
    np.savez_compressed(os.path.join(HERE, "ref_host.npz"), **host)
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        np.savez_compressed(os.path.join(HERE, "ref_reorder.npz"), **reorder_fixtures(host, td))
    with open(os.path.join(HERE, "ref_config1.json"), "w") as f:
        json.dump(big_digest(), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
