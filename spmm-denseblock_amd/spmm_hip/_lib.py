"""ctypes binding of libspmm_hip.so (the C ABI declared in include/spmm_hip.h,
include/spmm_host.h, include/spmm_reorder.h and include/spmm_multi.h).

The library is built in-tree by ``make -C spmm-denseblock_amd lib`` (or
``__graft_entry__.build()``). There is no fallback: if the library is missing
every entry point raises, so a GPU run can never silently fall back to a CPU
or eager-PyTorch path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (c_longlong, POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t,
                    c_uint64, c_void_p)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(ROOT_DIR, "lib", "libspmm_hip.so")

# Status codes: numeric values of cusparseStatus_t (include/spmm_hip.h).
STATUS_NAMES = {
    0: "SUCCESS", 1: "NOT_INITIALIZED", 2: "ALLOC_FAILED", 3: "INVALID_VALUE",
    4: "ARCH_MISMATCH", 5: "MAPPING_ERROR", 6: "EXECUTION_FAILED", 7: "INTERNAL_ERROR",
    8: "MATRIX_TYPE_NOT_SUPPORTED", 9: "ZERO_PIVOT", 10: "NOT_SUPPORTED",
}
SUCCESS, NOT_INITIALIZED, ALLOC_FAILED, INVALID_VALUE = 0, 1, 2, 3
EXECUTION_FAILED, MATRIX_TYPE_NOT_SUPPORTED, NOT_SUPPORTED = 6, 8, 10

DIRECTION_ROW, DIRECTION_COLUMN = 0, 1
OPERATION_NON_TRANSPOSE, OPERATION_TRANSPOSE = 0, 1
ORDER_ROW, ORDER_COL = 0, 1
INDEX_BASE_ZERO, INDEX_BASE_ONE = 0, 1
CSR_NT_STREAMS = 1
CSR_SEQUENTIAL_ROWS = 2
HYBRID_FUSED = 1
HYBRID_TWO_LAUNCH = 2
HYBRID_SPLIT_BF16 = 4
BSR_DENSE_BLOCK_PRODUCT = 1
BSR_SMALL_GROUPED = 2
BUILD_TUNING = 1


class SpmmError(RuntimeError):
    """Raised for a non-SUCCESS status; ``.status`` holds the numeric code."""

    def __init__(self, status: int, where: str):
        self.status = status
        super().__init__(f"{where}: SPMM_STATUS_{STATUS_NAMES.get(status, status)}")


def check(status: int, where: str) -> None:
    if status != SUCCESS:
        raise SpmmError(status, where)


_P = c_void_p
_PI = POINTER(c_int)
# name -> (restype, argtypes)
_PROTOS = {
    "spmm_get_version": (c_int, []),
    "spmm_get_status_string": (c_char_p, [c_int]),
    "spmm_create": (c_int, [POINTER(c_void_p)]),
    "spmm_destroy": (c_int, [_P]),
    "spmm_set_stream": (c_int, [_P, _P]),
    "spmm_get_stream": (c_int, [_P, POINTER(c_void_p)]),
    "spmm_create_mat_descr": (c_int, [POINTER(c_void_p)]),
    "spmm_destroy_mat_descr": (c_int, [_P]),
    "spmm_set_mat_type": (c_int, [_P, c_int]),
    "spmm_set_mat_index_base": (c_int, [_P, c_int]),
    "spmm_set_kernel_timing": (c_int, [_P, c_int]),
    "spmm_get_kernel_times": (c_int, [_P, POINTER(c_float), c_int, _PI]),
    "spmm_set_csr_waves_per_cu": (c_int, [_P, c_int]),
    "spmm_csr_default_waves_per_cu": (c_int, [c_int, c_int]),
    "spmm_set_csr_options": (c_int, [_P, c_int]),
    "spmm_set_hybrid_options": (c_int, [_P, c_int]),
    "spmm_set_bsr_options": (c_int, [_P, c_int]),
    "spmm_get_build_options": (c_int, []),
    "spmm_bsr_small_path": (c_int, [c_void_p, c_void_p]),
    "spmm_gespmm_csrmm_f32": (c_int, [c_int, c_int, _P, _P, _P, _P, _P, _P]),
    "spmm_scsrmm": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, POINTER(c_float), _P,
                            _P, _P, _P, _P, c_int, POINTER(c_float), _P, c_int]),
    "spmm_scsrmm2": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, POINTER(c_float), _P,
                             _P, _P, _P, _P, c_int, POINTER(c_float), _P, c_int]),
    "spmm_csrmm_ex_f32": (c_int, [_P, c_int, c_int, c_int, c_int, c_float, _P, _P, _P, c_int,
                                  _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_csr_hot_analysis": (c_int, [_P, c_int, c_int, c_int, _P, c_int, c_longlong, _P]),
    "spmm_csrmm_hot_f32": (c_int, [_P, c_int, c_int, c_int, c_int, c_float, _P, _P, _P, c_int,
                                   _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_sbsrmm": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            POINTER(c_float), _P, _P, _P, _P, c_int, _P, c_int,
                            POINTER(c_float), _P, c_int]),
    "spmm_bsrmm_ex_f32": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, _P, _P,
                                  _P, _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_bsrmm_ex_f16": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, _P, _P,
                                  _P, _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_bsr32_analysis_f32": (c_int, [_P, c_int, c_int, _P, _P, _P]),
    "spmm_bsrmm_analysed_f32": (c_int, [_P, c_int, c_int, c_int, c_int, c_float, _P, _P, _P, _P,
                                        _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_bsr16_analysis_f16": (c_int, [_P, c_int, c_int, _P, _P, _P]),
    "spmm_bsr16_group_analysis_f16": (c_int, [_P, c_int, c_int, c_int, c_int, _P, _P, _P, _P,
                                              POINTER(c_size_t)]),
    "spmm_bsrmm_grouped_f16": (c_int, [_P, c_int, c_int, c_int, _P, c_float, _P, c_int, c_int,
                                       c_float, _P, c_int, c_int]),
    "spmm_bsr16_group_release": (c_int, [_P, _P]),
    "spmm_bsr_group_release": (c_int, [_P, _P]),
    "spmm_bsr32_group_analysis_f32": (c_int, [_P, c_int, c_int, c_int, c_int, _P, _P, _P, _P,
                                              POINTER(c_size_t)]),
    "spmm_bsrmm_grouped_f32": (c_int, [_P, c_int, c_int, c_int, _P, c_float, _P, c_int, c_int,
                                       c_float, _P, c_int, c_int]),
    "spmm_bsrmm_analysed_f16": (c_int, [_P, c_int, c_int, c_int, c_int, c_float, _P, _P, _P, _P,
                                        _P, c_int, c_int, c_float, _P, c_int, c_int]),
    "spmm_gespmm_csrmm_f64": (c_int, [c_int, c_int, _P, _P, _P, _P, _P, _P]),
    "spmm_csrmm_ex_f64": (c_int, [_P, c_int, c_int, c_int, c_int, c_double, _P, _P, _P, c_int,
                                  _P, c_int, c_int, c_double, _P, c_int, c_int]),
    "spmm_dcsrmm2": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, POINTER(c_double), _P,
                             _P, _P, _P, _P, c_int, POINTER(c_double), _P, c_int]),
    "spmm_bsrmm_ex_f64": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_double, _P, _P,
                                  _P, _P, c_int, c_int, c_double, _P, c_int, c_int]),
    "spmm_dbsrmm": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            POINTER(c_double), _P, _P, _P, _P, c_int, _P, c_int,
                            POINTER(c_double), _P, c_int]),
    "spmm_xcsr2bsr_nnz": (c_int, [c_int, c_int, c_int, _P, _P, c_int, _P, _PI]),
    "spmm_scsr2bsr": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, _P]),
    "spmm_sbsr2csr": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, _P]),
    "spmm_calculate_nnzb": (c_int64, [c_int, _P, _P, c_int]),
    "spmm_csr_partition_rows": (c_int, [c_int, _P, c_int, _P]),
    "spmm_divide_nnz": (c_int, [c_int, _P, _P, c_int, c_float, _P, _P, _PI, _PI]),
    "spmm_sdivide": (c_int, [c_int, _P, _P, _P, c_int, c_float, _P, _P, _P, _P, _P, _P]),
    "spmm_xcsr2bsr_nnz_dev": (c_int, [_P, c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, _PI]),
    "spmm_xbsr_reblock32_nnzb": (c_int, [_P, c_int, c_int, c_int, c_int, _P, _P, _P, _PI]),
    "spmm_sbsr_reblock32": (c_int, [_P, c_int, c_int, c_int, c_int, _P, _P, _P, _P, c_int, _P,
                                    _P]),
    "spmm_scsr2bsr_dev": (c_int, [_P, c_int, c_int, c_int, _P, _P, _P, _P, c_int, _P, _P, _P,
                                  _P]),
    "spmm_sbsr2csr_dev": (c_int, [_P, c_int, c_int, c_int, _P, _P, _P, _P, c_int, _P, _P, _P,
                                  _P]),
    "spmm_xcoo2csr": (c_int, [_P, _P, c_int, c_int, _P, c_int]),
    # spmm_multi.h
    "spmm_multi_create": (c_int, [POINTER(c_void_p), c_int, _P]),
    "spmm_multi_destroy": (c_int, [_P]),
    "spmm_multi_size": (c_int, [_P]),
    "spmm_multi_get_stream": (c_int, [_P, c_int, POINTER(c_void_p)]),
    "spmm_multi_set_user_streams": (c_int, [_P, _P]),
    "spmm_multi_slot_rows": (c_int, [c_int, _P, c_int]),
    "spmm_csr_f32_multi": (c_int, [_P, c_int, c_int, c_int, _P, _P, _P, _P, _P, _P, c_int, _P,
                                   c_int, c_int]),
    "spmm_multi_synchronize": (c_int, [_P]),
    "spmm_multi_set_timing": (c_int, [_P, c_int]),
    "spmm_multi_get_times": (c_int, [_P, POINTER(c_float), POINTER(c_float)]),
    "spmm_hybrid_plan": (c_int, [c_int, _P, _P, c_int, c_int, c_int, c_double, c_double,
                                 POINTER(c_float), POINTER(c_int64), POINTER(c_int64),
                                 POINTER(c_double)]),
    "spmm_hybrid_csrmm_f32": (c_int, [_P, c_int, c_int, c_int, c_float, _P, _P, _P, c_int, c_int,
                                      _P, _P, _P, c_int, _P, c_int, c_float, _P, c_int]),
    "spmm_hybrid_csrmm_ex_f32": (c_int, [_P, c_int, c_int, c_int, c_float, _P, _P, _P, c_int,
                                         c_int, _P, _P, _P, c_int, _P, c_int, c_int, c_float, _P,
                                         c_int, c_int]),
    # spmm_host.h
    "spmm_host_free": (None, [_P]),
    "spmm_host_rng_seed": (None, [c_uint64]),
    "spmm_host_random_array": (None, [c_int64, c_float, c_float, _P]),
    "spmm_host_random_csr": (c_int64, [c_int, c_int, c_float, c_float, c_float, _P,
                                       POINTER(c_void_p), POINTER(c_void_p)]),
    "spmm_host_random_bsr": (c_int64, [c_int, c_int, c_int, c_float, c_float, c_float, _P,
                                       POINTER(c_void_p), POINTER(c_void_p)]),
    "spmm_host_dump_csr": (c_int, [c_char_p, c_int, c_int64, _P, _P]),
    "spmm_host_load_csr": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_void_p), _PI,
                                   POINTER(c_int64)]),
    "spmm_host_load_graph": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_void_p), _PI,
                                     POINTER(c_int64)]),
    "spmm_host_save_csr_bin": (c_int, [c_char_p, c_int, c_int64, _P, _P, _P]),
    "spmm_host_load_csr_bin": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_void_p),
                                       POINTER(c_void_p), _PI, POINTER(c_int64)]),
    "spmm_host_load_csr_cached": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_void_p), _PI,
                                          POINTER(c_int64)]),
    "spmm_host_gen_powerlaw_csr": (c_int, [c_int, c_int64, c_int, c_double, c_uint64,
                                           POINTER(c_void_p), POINTER(c_void_p)]),
    "spmm_host_gen_community_csr": (c_int, [c_int, c_double, c_int, c_int, c_double, c_uint64,
                                            POINTER(c_void_p), POINTER(c_void_p),
                                            POINTER(c_int64)]),
    # spmm_reorder.h
    "spmm_reorder_degree": (c_int, [c_int, _P, _P, _P]),
    "spmm_reorder_bfs": (c_int, [c_int, _P, _P, _P]),
    "spmm_reorder_rcm": (c_int, [c_int, _P, _P, _P]),
    "spmm_permute_csr": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P]),
    "spmm_check_permutation": (c_int, [c_int, _P]),
    "spmm_load_permutation": (c_int, [c_char_p, c_int, _P]),
    "spmm_dump_permutation": (c_int, [c_char_p, c_int, _P]),
    "spmm_block_metrics": (c_int, [c_int, _P, _P, c_int, _P]),
    "spmm_block_heatmap": (c_int, [c_int, _P, _P, c_int, _P]),
    "spmm_dump_heatmap": (c_int, [c_char_p, c_int, _P]),
}


class BlockMetrics(ctypes.Structure):
    """spmm_block_metrics_t (include/spmm_reorder.h)."""
    _fields_ = [("block_dim", c_int), ("nnzb", c_int64), ("density", c_double),
                ("utilization", c_double), ("average", c_double)]


# Symbols every build must export (tests/test_abi.py checks them against the
# headers too).
EXPORTED = tuple(_PROTOS)

_lib = None


def lib() -> ctypes.CDLL:
    """Load libspmm_hip.so once; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libspmm_hip.so not found at {LIB_PATH}: the HIP extension is not built "
                "(run `make -C spmm-denseblock_amd lib` or __graft_entry__.build()). "
                "There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib
