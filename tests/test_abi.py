"""The C-ABI library loads and exports every symbol include/*.h declares, the
Python binding covers them, and argument checking that happens before any
device work behaves as documented. CPU only (no compute calls)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared() -> set[str]:
    names = set()
    for h in ("spmm_hip.h", "spmm_host.h", "spmm_reorder.h", "spmm_multi.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(spmm_[a-z0-9_]+)\s*\(", src))
    return names


def test_headers_declare_the_boundary():
    d = _declared()
    for must in ("spmm_gespmm_csrmm_f32", "spmm_scsrmm", "spmm_scsrmm2", "spmm_sbsrmm",
                 "spmm_csrmm_ex_f32", "spmm_bsrmm_ex_f32", "spmm_bsrmm_ex_f16",
                 "spmm_xcsr2bsr_nnz", "spmm_scsr2bsr", "spmm_sbsr2csr", "spmm_calculate_nnzb",
                 "spmm_csr_partition_rows", "spmm_xcoo2csr", "spmm_csr_f32_multi",
                 "spmm_multi_create"):
        assert must in d


def test_library_exports_every_declared_symbol():
    from spmm_hip import _lib
    so = _lib.LIB_PATH
    assert os.path.exists(so), "libspmm_hip.so not built"
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = _declared() - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    assert _declared() <= set(_lib.EXPORTED), "binding misses declared symbols"
    L = _lib.lib()
    assert L.spmm_get_version() == 100


def test_gfx950_code_object_present():
    """The fat binary embeds an amdgcn gfx950 code object (and no other ISA)."""
    from spmm_hip import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"amdgcn-amd-amdhsa--gfx906" not in data


def test_status_strings_and_host_side_checks():
    from spmm_hip import _lib
    L = _lib.lib()
    assert L.spmm_get_status_string(3) == b"SPMM_STATUS_INVALID_VALUE"
    assert L.spmm_get_status_string(8) == b"SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED"
    # Argument errors are reported before any device work (no GPU needed).
    assert L.spmm_gespmm_csrmm_f32(-1, 4, None, None, None, None, None, None) == 3
    assert L.spmm_gespmm_csrmm_f32(0, 4, None, None, None, None, None, None) == 0  # quick return
    assert L.spmm_gespmm_csrmm_f32(4, 4, None, None, None, None, None, None) == 3
    one = ctypes.c_float(1.0)
    assert L.spmm_sbsrmm(None, 0, 0, 0, 1, 1, 1, 1, ctypes.byref(one), None, None, None, None, 2,
                         None, 1, ctypes.byref(one), None, 1) == 1  # NOT_INITIALIZED
    assert L.spmm_csrmm_ex_f32(None, 1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0, None,
                               1, 0) == 1
    # multi-GPU context: argument checks and the partition helper need no GPU
    assert L.spmm_multi_destroy(None) == 1
    assert L.spmm_multi_create(None, 1, None) == 3
    assert L.spmm_csr_f32_multi(None, 4, 4, 4, None, None, None, None, None, None, 4, None, 4,
                                1) == 1
    b = (ctypes.c_int * 4)(0, 5, 9, 10)
    assert L.spmm_multi_slot_rows(3, b, 1) == 5
    assert L.spmm_multi_slot_rows(3, b, 2) == 3
    assert L.spmm_multi_slot_rows(3, b, 0) == 0
    assert L.spmm_xcoo2csr(None, None, 0, 0, None, 0) == 1
    # the bs 32 analysis entries: a null handle is NOT_INITIALIZED before anything else
    assert L.spmm_bsr32_analysis_f32(None, 0, 4, None, None, None) == 1
    assert L.spmm_bsrmm_analysed_f32(None, 1, 1, 4, 1, 1.0, None, None, None, None, None, 4, 0,
                                     0.0, None, 4, 0) == 1
    # the hot-column CSR entries likewise
    assert L.spmm_csr_hot_analysis(None, 128, 4, 4, None, 0, 0, None) == 1
    assert L.spmm_csrmm_hot_f32(None, 1, 1, 1, 0, 1.0, None, None, None, 0, None, 1, 0, 0.0,
                                None, 1, 0) == 1
    # the CSR grid's default target (host-only): 12 waves per CU from 2^20 rows on the
    # plain kernel, 16 below and for the hot-column kernel; bench.py reports it
    assert L.spmm_csr_default_waves_per_cu(2449029, 0) == 12
    assert L.spmm_csr_default_waves_per_cu((1 << 20) - 1, 0) == 16
    assert L.spmm_csr_default_waves_per_cu(2449029, 1) == 16
    assert L.spmm_csr_default_waves_per_cu(169343, 0) == 16
    d = ctypes.c_void_p()
    assert L.spmm_create_mat_descr(ctypes.byref(d)) == 0
    assert L.spmm_set_mat_index_base(d, 1) == 0
    assert L.spmm_set_mat_index_base(d, 7) == 3
    assert L.spmm_destroy_mat_descr(d) == 0


def test_release_build_reads_no_environment():
    """The shipped library is a release build: its kernel choice cannot be
    changed by SPMM_BSR_VARIANT / SPMM_BSR_ORDER / SPMM_CSR_GROUP_PD (those
    are read only by a `make TUNING=1` A/B build), and the binary names none
    of them."""
    from spmm_hip import _lib
    L = _lib.lib()
    assert L.spmm_get_build_options() & _lib.BUILD_TUNING == 0
    data = open(_lib.LIB_PATH, "rb").read()
    for var in (b"SPMM_BSR_VARIANT", b"SPMM_BSR_ORDER", b"SPMM_CSR_GROUP_PD", b"SPMM_GRP_VARIANT",
                b"SPMM_CSR_MIN_ITEMS", b"SPMM_GRP32_VARIANT", b"SPMM_GRP_XM", b"SPMM_GRP_TT",
                b"SPMM_CS16_TT", b"SPMM_SMALL_XM"):
        assert var not in data, var
    assert L.spmm_set_bsr_options(None, 1) == 1
    assert L.spmm_get_version() == 100


def test_no_silent_fallback_when_library_missing(monkeypatch):
    from spmm_hip import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libspmm_hip.so")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()
