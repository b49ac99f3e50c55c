"""Host-side preprocessing and data feeders (numpy in, numpy out).

Thin wrappers over the C ABI of libspmm_hip.so:
  csr2bsr / bsr2csr / calculate_nnzb / partition_rows   (include/spmm_hip.h)
  rng_seed / random_array / random_csr / random_bsr /
  load_csr / dump_csr / load_graph / save_csr_bin / load_csr_bin / load_csr_cached /
  powerlaw_csr / community_csr                                  (include/spmm_host.h)
  reorder / permute_csr / load_permutation / dump_permutation /
  block_metrics / block_heatmap / dump_heatmap                  (include/spmm_reorder.h)
All conversion work happens in the library's C++ (north_star: CPU-side
preprocessing), not in Python.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_int64, c_void_p

import numpy as np

from ._lib import BlockMetrics, check, lib


def _p(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data) if a is not None and a.size else c_void_p(0)


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _take(ptr: c_void_p, n: int, dtype) -> np.ndarray:
    """Copy n elements from a malloc'ed C array and free it."""
    if not ptr.value:
        raise MemoryError("libspmm_hip returned a null array")
    if n:
        buf = (ctypes.c_byte * (n * np.dtype(dtype).itemsize)).from_address(ptr.value)
        out = np.frombuffer(buf, dtype=dtype).copy()
    else:
        out = np.zeros(0, dtype=dtype)
    lib().spmm_host_free(ptr)
    return out


# --------------------------------------------------------------- conversions
def csr2bsr(m: int, n: int, rowptr, colind, val, bs: int, direction: int = 0):
    """cusparseXcsr2bsrNnz + cusparseScsr2bsr semantics (run_bsrmm.cu:116-142).
    Returns (bsr_rowptr[mb+1], bsr_colind[nnzb], bsr_val[nnzb*bs*bs])."""
    rowptr, colind, val = _i32(rowptr), _i32(colind), _f32(val)
    mb = (m + bs - 1) // bs
    brp = np.zeros(mb + 1, dtype=np.int32)
    nnzb = c_int(0)
    check(lib().spmm_xcsr2bsr_nnz(direction, m, n, _p(rowptr), _p(colind), bs, _p(brp),
                                  byref(nnzb)), "spmm_xcsr2bsr_nnz")
    bci = np.zeros(nnzb.value, dtype=np.int32)
    bval = np.zeros(nnzb.value * bs * bs, dtype=np.float32)
    check(lib().spmm_scsr2bsr(direction, m, n, _p(val), _p(rowptr), _p(colind), bs, _p(brp),
                              _p(bval), _p(bci)), "spmm_scsr2bsr")
    return brp, bci, bval


def bsr2csr(mb: int, nb: int, rowptr, colind, val, bs: int, direction: int = 0):
    """cusparseSbsr2csr semantics (bsr2csr.cu:177-188): nnz = nnzb*bs*bs."""
    rowptr, colind, val = _i32(rowptr), _i32(colind), _f32(val)
    nnz = int(rowptr[-1] - rowptr[0]) * bs * bs
    rp = np.zeros(mb * bs + 1, dtype=np.int32)
    ci = np.zeros(nnz, dtype=np.int32)
    v = np.zeros(nnz, dtype=np.float32)
    check(lib().spmm_sbsr2csr(direction, mb, nb, _p(val), _p(rowptr), _p(colind), bs, _p(v),
                              _p(rp), _p(ci)), "spmm_sbsr2csr")
    return rp, ci, v


def calculate_nnzb(n: int, rowptr, colind, bs: int) -> int:
    """calculateNnzb (utility.cc:47-69)."""
    rowptr, colind = _i32(rowptr), _i32(colind)
    r = lib().spmm_calculate_nnzb(n, _p(rowptr), _p(colind), bs)
    if r < 0:
        raise ValueError("spmm_calculate_nnzb: invalid input")
    return int(r)


def divide(n: int, rowptr, colind, val, bs: int, density: float):
    """divide_matrix (divide.cu:52-127) with values: blocks with fill >= density
    -> BSR (DIRECTION_ROW), the rest -> CSR remainder. Returns
    (csr_rowptr, csr_colind, csr_val, bsr_rowptr, bsr_colind, bsr_val)."""
    rowptr, colind, val = _i32(rowptr), _i32(colind), _f32(val)
    mb = (n + bs - 1) // bs
    crp = np.zeros(n + 1, dtype=np.int32)
    brp = np.zeros(mb + 1, dtype=np.int32)
    cn, nb = c_int(0), c_int(0)
    check(lib().spmm_divide_nnz(n, _p(rowptr), _p(colind), bs, density, _p(crp), _p(brp),
                                byref(cn), byref(nb)), "spmm_divide_nnz")
    cci = np.zeros(cn.value, dtype=np.int32)
    cv = np.zeros(cn.value, dtype=np.float32)
    bci = np.zeros(nb.value, dtype=np.int32)
    bv = np.zeros(nb.value * bs * bs, dtype=np.float32)
    check(lib().spmm_sdivide(n, _p(rowptr), _p(colind), _p(val), bs, density, _p(crp), _p(brp),
                             _p(cci), _p(cv), _p(bci), _p(bv)), "spmm_sdivide")
    return crp, cci, cv, brp, bci, bv


def hybrid_plan(rowptr, colind, bs: int, K: int, value_bytes: int = 4,
                bsr_bytes_per_s: float = 0.0, csr_bytes_per_s: float = 0.0) -> dict:
    """spmm_hybrid_plan: the divide density threshold minimising the modelled
    hybrid time. Returns {density, nnzb, csr_nnz, est_seconds}."""
    from ctypes import c_double, c_float
    rowptr, colind = _i32(rowptr), _i32(colind)
    d, nb, cn, est = c_float(0), c_int64(0), c_int64(0), c_double(0)
    check(lib().spmm_hybrid_plan(rowptr.size - 1, _p(rowptr), _p(colind), bs, K, value_bytes,
                                 bsr_bytes_per_s, csr_bytes_per_s, byref(d), byref(nb),
                                 byref(cn), byref(est)), "spmm_hybrid_plan")
    return {"density": d.value, "nnzb": nb.value, "csr_nnz": cn.value,
            "est_seconds": est.value}


def partition_rows(rowptr, nparts: int) -> np.ndarray:
    """nnz-balanced contiguous row split: bounds[nparts+1]."""
    rowptr = _i32(rowptr)
    b = np.zeros(nparts + 1, dtype=np.int32)
    check(lib().spmm_csr_partition_rows(rowptr.size - 1, _p(rowptr), nparts, _p(b)),
          "spmm_csr_partition_rows")
    return b


# -------------------------------------------------------------- data feeders
def rng_seed(seed: int = 1234) -> None:
    lib().spmm_host_rng_seed(seed)


def random_array(n: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """randomArray (load_data.cc:29-36) from the shared mt19937_64."""
    out = np.empty(n, dtype=np.float32)
    lib().spmm_host_random_array(n, lo, hi, _p(out))
    return out


def random_dense_matrix(n: int, dim: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """randomDenseMatrix (load_data.cc:38-40), returned as (n, dim) row-major."""
    return random_array(n * dim, lo, hi).reshape(n, dim)


def random_csr(m: int, n: int, p: float, lo: float = -1.0, hi: float = 1.0):
    """randomCSRMatrix (load_data.cc:42-69) -> (rowptr, colind, val)."""
    rp = np.zeros(m + 1, dtype=np.int32)
    ci, v = c_void_p(), c_void_p()
    nnz = lib().spmm_host_random_csr(m, n, p, lo, hi, _p(rp), byref(ci), byref(v))
    if nnz < 0:
        raise ValueError("spmm_host_random_csr failed")
    return rp, _take(ci, nnz, np.int32), _take(v, nnz, np.float32)


def random_bsr(mb: int, nb: int, bs: int, p: float, lo: float = -1.0, hi: float = 1.0):
    """randomBSRMatrix (load_data.cc:81-113) -> (rowptr, colind, val)."""
    rp = np.zeros(mb + 1, dtype=np.int32)
    ci, v = c_void_p(), c_void_p()
    nnzb = lib().spmm_host_random_bsr(mb, nb, bs, p, lo, hi, _p(rp), byref(ci), byref(v))
    if nnzb < 0:
        raise ValueError("spmm_host_random_bsr failed")
    return rp, _take(ci, nnzb, np.int32), _take(v, nnzb * bs * bs, np.float32)


def dump_csr(prefix: str, rowptr, colind) -> None:
    rowptr, colind = _i32(rowptr), _i32(colind)
    if lib().spmm_host_dump_csr(prefix.encode(), rowptr.size - 1, colind.size, _p(rowptr),
                                _p(colind)) != 0:
        raise OSError(f"dump_csr({prefix}) failed")


def load_csr(prefix: str):
    """loadCSRFromFile (load_data.cc:143-165) -> (rowptr, colind)."""
    rp, ci, n, nnz = c_void_p(), c_void_p(), c_int(0), c_int64(0)
    if lib().spmm_host_load_csr(prefix.encode(), byref(rp), byref(ci), byref(n), byref(nnz)) != 0:
        raise OSError(f"load_csr({prefix}) failed")
    return _take(rp, n.value + 1, np.int32), _take(ci, nnz.value, np.int32)


def save_csr_bin(path: str, rowptr, colind, val=None) -> None:
    """Binary sidecar (magic SPMMCSR1 + per-array checksums), include/spmm_host.h."""
    rowptr, colind = _i32(rowptr), _i32(colind)
    v = None if val is None else _f32(val)
    if lib().spmm_host_save_csr_bin(path.encode(), rowptr.size - 1, colind.size, _p(rowptr),
                                    _p(colind), None if v is None else _p(v)) != 0:
        raise OSError(f"save_csr_bin({path}) failed")


def load_csr_bin(path: str):
    """-> (rowptr, colind, val or None); raises on a missing or corrupt file."""
    rp, ci, v, n, nnz = c_void_p(), c_void_p(), c_void_p(), c_int(0), c_int64(0)
    rc = lib().spmm_host_load_csr_bin(path.encode(), byref(rp), byref(ci), byref(v), byref(n),
                                      byref(nnz))
    if rc == -2:
        raise ValueError(f"load_csr_bin({path}): checksum mismatch (corrupt cache)")
    if rc != 0:
        raise OSError(f"load_csr_bin({path}) failed")
    vals = _take(v, nnz.value, np.float32) if v.value else None
    return _take(rp, n.value + 1, np.int32), _take(ci, nnz.value, np.int32), vals


def load_csr_cached(prefix: str):
    """loadCSRFromFile through <prefix>.csrbin (used when fresh and intact,
    rewritten otherwise) -> (rowptr, colind)."""
    rp, ci, n, nnz = c_void_p(), c_void_p(), c_int(0), c_int64(0)
    if lib().spmm_host_load_csr_cached(prefix.encode(), byref(rp), byref(ci), byref(n),
                                       byref(nnz)) != 0:
        raise OSError(f"load_csr_cached({prefix}) failed")
    return _take(rp, n.value + 1, np.int32), _take(ci, nnz.value, np.int32)


def load_graph(filename: str):
    """loadGraphFromFile (load_data.cc:167-184) + convertGraphToCSR."""
    rp, ci, n, nnz = c_void_p(), c_void_p(), c_int(0), c_int64(0)
    if lib().spmm_host_load_graph(filename.encode(), byref(rp), byref(ci), byref(n),
                                  byref(nnz)) != 0:
        raise OSError(f"load_graph({filename}) failed")
    return _take(rp, n.value + 1, np.int32), _take(ci, nnz.value, np.int32)


def powerlaw_csr(n: int, nnz: int, max_deg: int, gamma: float = 2.3, seed: int = 1234):
    """Chung-Lu power-law stand-in for an OGB graph (include/spmm_host.h)."""
    rp, ci = c_void_p(), c_void_p()
    if lib().spmm_host_gen_powerlaw_csr(n, nnz, max_deg, gamma, seed, byref(rp), byref(ci)) != 0:
        raise ValueError("spmm_host_gen_powerlaw_csr: invalid parameters")
    return _take(rp, n + 1, np.int32), _take(ci, nnz, np.int32)


def community_csr(n: int, avg_deg: float, cmin: int, cmax: int, p_in: float, seed: int = 1234):
    """Community-ordered stand-in for a rabbit-reordered graph (include/spmm_host.h)."""
    rp, ci, nnz = c_void_p(), c_void_p(), c_int64(0)
    if lib().spmm_host_gen_community_csr(n, avg_deg, cmin, cmax, p_in, seed, byref(rp), byref(ci),
                                         byref(nnz)) != 0:
        raise ValueError("spmm_host_gen_community_csr: invalid parameters")
    return _take(rp, n + 1, np.int32), _take(ci, nnz.value, np.int32)


# ------------------------------------------------------- reorder front-end
_REORDER = {"degree": "spmm_reorder_degree", "bfs": "spmm_reorder_bfs",
            "rcm": "spmm_reorder_rcm"}


def _ok(rc: int, where: str) -> None:
    if rc != 0:
        raise ValueError(f"{where}: invalid input")


def reorder(rowptr, colind, method: str = "rcm") -> np.ndarray:
    """old2new permutation: "degree" (maxDegreeSort, reorder_strategy.cc:57-71),
    "bfs" (BFSTraversal, :84-114) or "rcm" (reverseCuthillMcKee, :73-82)."""
    if method not in _REORDER:
        raise ValueError(f"unknown reorder method {method!r}; choose from {sorted(_REORDER)}")
    rowptr, colind = _i32(rowptr), _i32(colind)
    out = np.empty(rowptr.size - 1, dtype=np.int32)
    _ok(getattr(lib(), _REORDER[method])(rowptr.size - 1, _p(rowptr), _p(colind), _p(out)),
        _REORDER[method])
    return out


def permute_csr(rowptr, colind, old2new, val=None):
    """permutate (reorder_strategy.cc:42-55): symmetric renumbering with sorted
    columns; values follow their columns. Returns (rowptr, colind[, val])."""
    rowptr, colind, old2new = _i32(rowptr), _i32(colind), _i32(old2new)
    n = rowptr.size - 1
    nrp = np.empty(n + 1, dtype=np.int32)
    nci = np.empty(colind.size, dtype=np.int32)
    if val is None:
        _ok(lib().spmm_permute_csr(n, _p(rowptr), _p(colind), None, _p(old2new), _p(nrp),
                                   _p(nci), None), "spmm_permute_csr")
        return nrp, nci
    val = _f32(val)
    nv = np.empty(val.size, dtype=np.float32)
    _ok(lib().spmm_permute_csr(n, _p(rowptr), _p(colind), _p(val), _p(old2new), _p(nrp),
                               _p(nci), _p(nv)), "spmm_permute_csr")
    return nrp, nci, nv


def load_permutation(filename: str, n: int) -> np.ndarray:
    """loadPermutation (rabbit_reorder.cc:10-19), validated as a permutation."""
    out = np.empty(n, dtype=np.int32)
    if lib().spmm_load_permutation(filename.encode(), n, _p(out)) != 0:
        raise ValueError(f"load_permutation({filename}): unreadable or not a permutation of {n}")
    return out


def dump_permutation(filename: str, old2new) -> None:
    old2new = _i32(old2new)
    if lib().spmm_dump_permutation(filename.encode(), old2new.size, _p(old2new)) != 0:
        raise OSError(f"dump_permutation({filename}) failed")


def block_metrics(rowptr, colind, bs: int) -> dict:
    """analyzeBlockSparseMetrics (reorder_graph.cc:12-24) at one block size."""
    rowptr, colind = _i32(rowptr), _i32(colind)
    m = BlockMetrics()
    _ok(lib().spmm_block_metrics(rowptr.size - 1, _p(rowptr), _p(colind), bs,
                                 c_void_p(ctypes.addressof(m))), "spmm_block_metrics")
    return {"block_dim": m.block_dim, "nnzb": m.nnzb, "density": m.density,
            "utilization": m.utilization, "average": m.average}


def block_heatmap(rowptr, colind, bs: int) -> np.ndarray:
    """getHeatmap (utility.cc:71-88): nnz per bs x bs block, shape (nb, nb)."""
    rowptr, colind = _i32(rowptr), _i32(colind)
    n = rowptr.size - 1
    nb = (n + bs - 1) // bs
    out = np.empty(nb * nb, dtype=np.int32)
    _ok(lib().spmm_block_heatmap(n, _p(rowptr), _p(colind), bs, _p(out)), "spmm_block_heatmap")
    return out.reshape(nb, nb)


def dump_heatmap(filename: str, heatmap) -> None:
    """dumpHeatmap (utility.cc:90-100) text format."""
    h = np.ascontiguousarray(heatmap, dtype=np.int32)
    if h.ndim != 2 or h.shape[0] != h.shape[1]:
        raise ValueError("heatmap must be square")
    if lib().spmm_dump_heatmap(filename.encode(), h.shape[0], _p(h)) != 0:
        raise OSError(f"dump_heatmap({filename}) failed")
