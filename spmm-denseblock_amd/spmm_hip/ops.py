"""Device SpMM entry points over torch tensors (HIP memory + streams only).

torch is plumbing here: it owns the device buffers and the stream; every
FLOP runs in the hand-written gfx950 kernels of libspmm_hip.so, called
through the C ABI. The functions mirror the reference's operator interfaces:

  gespmm_csrmm(...)   gespmm_csrmm<float>(A_nrows, B_ncols, rowPtr, colInd, val, B, C)
                      (gespmm_csrmm.h:422-426): C = A*B, row-major, overwritten
  csrmm(...)          cusparseScsrmm / csrmm2 with explicit storage orders
  bsrmm(...)          cusparseSbsrmm / rocsparse_bsrmm_template<float>
  bsrmm_f16(...)      fp16 A/B, fp32 accumulate (config 5)
"""
from __future__ import annotations

from ctypes import byref, c_float, c_int, c_void_p

import torch

from ._lib import (DIRECTION_ROW, ORDER_COL, ORDER_ROW, SpmmError, check, lib)


def _ptr(t: torch.Tensor | None) -> c_void_p:
    return c_void_p(t.data_ptr() if t is not None and t.numel() else 0)


def _need(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must live on a HIP device (there is no CPU path)")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class Handle:
    """spmm_handle_t bound to a torch stream (default: the current stream)."""

    def __init__(self, stream: torch.cuda.Stream | None = None):
        h = c_void_p()
        check(lib().spmm_create(byref(h)), "spmm_create")
        self._h = h
        self.set_stream(stream if stream is not None else torch.cuda.current_stream())

    @property
    def raw(self) -> c_void_p:
        return self._h

    def set_stream(self, stream: torch.cuda.Stream) -> None:
        self.stream = stream
        check(lib().spmm_set_stream(self._h, c_void_p(stream.cuda_stream)), "spmm_set_stream")

    def set_timing(self, enable: bool) -> None:
        check(lib().spmm_set_kernel_timing(self._h, int(enable)), "spmm_set_kernel_timing")

    def kernel_times(self, max_count: int = 1 << 16) -> list[float]:
        """Durations (ms) of every main-kernel launch since the last call,
        measured with hipEvents on the handle's stream."""
        buf = (c_float * max_count)()
        cnt = c_int(0)
        check(lib().spmm_get_kernel_times(self._h, buf, max_count, byref(cnt)),
              "spmm_get_kernel_times")
        return list(buf[: cnt.value])

    def set_csr_waves_per_cu(self, w: int) -> None:
        check(lib().spmm_set_csr_waves_per_cu(self._h, w), "spmm_set_csr_waves_per_cu")

    def set_csr_options(self, flags: int) -> None:
        check(lib().spmm_set_csr_options(self._h, flags), "spmm_set_csr_options")

    def set_hybrid_options(self, flags: int) -> None:
        check(lib().spmm_set_hybrid_options(self._h, flags), "spmm_set_hybrid_options")

    def set_bsr_options(self, flags: int) -> None:
        check(lib().spmm_set_bsr_options(self._h, flags), "spmm_set_bsr_options")

    def small_bsr_path(self) -> int:
        """spmm_bsr_small_path: the kernel of the last bs 2 / 4 / 8 fp32 product
        (0 lane-group VALU, 1 grouped MFMA stream, 2 grouped branch given up by
        its probe, -1 none). Synchronises the handle's stream."""
        from ctypes import byref, c_int
        p = c_int(-1)
        check(lib().spmm_bsr_small_path(self._h, byref(p)), "spmm_bsr_small_path")
        return p.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().spmm_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_handles: dict[int, Handle] = {}


def default_handle() -> Handle:
    dev = torch.cuda.current_device()
    h = _handles.get(dev)
    if h is None:
        h = _handles[dev] = Handle()
    h.set_stream(torch.cuda.current_stream())
    return h


_SUFFIX = {torch.float32: "f32", torch.float64: "f64"}


def _value_type(val: torch.Tensor) -> torch.dtype:
    """fp32 or fp64 (the T of gespmm_csrmm<T> / rocsparse_bsrmm_template<T>)."""
    if val.dtype not in _SUFFIX:
        raise TypeError(f"val must be float32 or float64, got {val.dtype}")
    return val.dtype


def gespmm_csrmm(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor,
                 B: torch.Tensor, C: torch.Tensor | None = None) -> torch.Tensor:
    """Drop-in for gespmm_csrmm<T> (gespmm_csrmm.h:422-426), T = float or double
    from val's dtype. rowptr int32[m+1], colind int32[nnz], val T[nnz], B T[k, K]
    row-major; returns C T[m, K] (overwritten, no alpha/beta)."""
    dt = _value_type(val)
    for t, d, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                     (val, dt, "val"), (B, dt, "B")):
        _need(t, d, nm)
    m = rowptr.numel() - 1
    K = B.shape[1]
    if C is None:
        C = torch.empty((m, K), dtype=dt, device=B.device)
    _need(C, dt, "C")
    if C.shape != (m, K):
        raise ValueError(f"C must be {(m, K)}, got {tuple(C.shape)}")
    fn = "spmm_gespmm_csrmm_" + _SUFFIX[dt]
    check(getattr(lib(), fn)(m, K, _ptr(rowptr), _ptr(colind), _ptr(val), _ptr(B), _ptr(C),
                             c_void_p(torch.cuda.current_stream().cuda_stream)), fn)
    return C


def csrmm(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, B: torch.Tensor, *,
          m: int | None = None, n: int, k: int, ldb: int, order_b: int = ORDER_ROW,
          C: torch.Tensor, ldc: int, order_c: int = ORDER_ROW, alpha: float = 1.0,
          beta: float = 0.0, base: int = 0, handle: Handle | None = None) -> torch.Tensor:
    """C(m x n) = alpha * A(m x k, csr) * B(k x n) + beta * C with explicit
    storage orders and leading dimensions (spmm_csrmm_ex_f32 / _f64 by val's dtype)."""
    dt = _value_type(val)
    for t, d, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                     (val, dt, "val"), (B, dt, "B"), (C, dt, "C")):
        _need(t, d, nm)
    h = handle or default_handle()
    m = rowptr.numel() - 1 if m is None else m
    fn = "spmm_csrmm_ex_" + _SUFFIX[dt]
    check(getattr(lib(), fn)(h.raw, m, n, k, colind.numel(), alpha, _ptr(rowptr), _ptr(colind),
                             _ptr(val), base, _ptr(B), ldb, order_b, beta, _ptr(C), ldc,
                             order_c), fn)
    return C


def csr_hot_analysis(colind: torch.Tensor, *, n: int, k: int, base: int = 0,
                     hot_bytes: int = 0, out: torch.Tensor | None = None,
                     handle: Handle | None = None) -> torch.Tensor:
    """spmm_csr_hot_analysis: colind with bit 31 set on the hot columns (the
    most used B rows whose n-float pieces fit in hot_bytes; 0 = the library
    default). Once per matrix; feed the result to csrmm_hot."""
    _need(colind, torch.int32, "colind")
    if out is None:
        out = torch.empty_like(colind)
    _need(out, torch.int32, "out")
    if out.numel() < colind.numel():
        raise ValueError("out is shorter than colind")
    h = handle or default_handle()
    check(lib().spmm_csr_hot_analysis(h.raw, n, k, colind.numel(), _ptr(colind), base, hot_bytes,
                                      _ptr(out)), "spmm_csr_hot_analysis")
    return out


def csrmm_hot(rowptr: torch.Tensor, colind_hot: torch.Tensor, val: torch.Tensor,
              B: torch.Tensor, *, m: int | None = None, n: int, k: int, ldb: int,
              order_b: int = ORDER_ROW, C: torch.Tensor, ldc: int, order_c: int = ORDER_ROW,
              alpha: float = 1.0, beta: float = 0.0, base: int = 0,
              handle: Handle | None = None) -> torch.Tensor:
    """csrmm on the tagged indices of csr_hot_analysis (spmm_csrmm_hot_f32):
    the same result, bit for bit, with cache hints on the B-row gathers."""
    for t, d, nm in ((rowptr, torch.int32, "rowptr"), (colind_hot, torch.int32, "colind_hot"),
                     (val, torch.float32, "val"), (B, torch.float32, "B"),
                     (C, torch.float32, "C")):
        _need(t, d, nm)
    h = handle or default_handle()
    m = rowptr.numel() - 1 if m is None else m
    check(lib().spmm_csrmm_hot_f32(h.raw, m, n, k, colind_hot.numel(), alpha, _ptr(rowptr),
                                   _ptr(colind_hot), _ptr(val), base, _ptr(B), ldb, order_b, beta,
                                   _ptr(C), ldc, order_c), "spmm_csrmm_hot_f32")
    return C


def bsrmm(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, B: torch.Tensor, *,
          mb: int, kb: int, n: int, bs: int, ldb: int, order_b: int = ORDER_ROW,
          C: torch.Tensor, ldc: int, order_c: int = ORDER_ROW, alpha: float = 1.0,
          beta: float = 0.0, direction: int = DIRECTION_ROW,
          handle: Handle | None = None) -> torch.Tensor:
    """C(mb*bs x n) = alpha * A(bsr) * B(kb*bs x n) + beta * C
    (spmm_bsrmm_ex_f32 / _f64 by val's dtype)."""
    dt = _value_type(val)
    for t, d, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                     (val, dt, "val"), (B, dt, "B"), (C, dt, "C")):
        _need(t, d, nm)
    h = handle or default_handle()
    fn = "spmm_bsrmm_ex_" + _SUFFIX[dt]
    check(getattr(lib(), fn)(h.raw, direction, mb, kb, n, colind.numel(), bs, alpha,
                             _ptr(rowptr), _ptr(colind), _ptr(val), _ptr(B), ldb, order_b, beta,
                             _ptr(C), ldc, order_c), fn)
    return C


def bsr32_analysis(val: torch.Tensor, *, nnzb: int, direction: int = DIRECTION_ROW,
                   masks: torch.Tensor | None = None, val_col: torch.Tensor | None = None,
                   handle: Handle | None = None):
    """Column masks of the bs = 32 blocks (int32 words, bit c = column c holds a
    value other than +-0) and, for ROW blocks, their column-major copy
    (spmm_bsr32_analysis_f32). Returns (masks, val_col); val_col is val itself
    for COLUMN blocks."""
    _need(val, torch.float32, "val")
    if val.numel() < nnzb * 1024:
        raise ValueError(f"val holds {val.numel()} floats, {nnzb} blocks need {nnzb * 1024}")
    if masks is None:
        masks = torch.empty(max(nnzb, 1), dtype=torch.int32, device=val.device)
    if direction == DIRECTION_ROW and val_col is None:
        val_col = torch.empty(max(nnzb, 1) * 1024, dtype=torch.float32, device=val.device)
    _need(masks, torch.int32, "masks")
    if masks.numel() < nnzb:
        raise ValueError("masks holds fewer than nnzb words")
    if direction == DIRECTION_ROW:
        _need(val_col, torch.float32, "val_col")
        if val_col.numel() < nnzb * 1024:
            raise ValueError("val_col holds fewer than nnzb * 1024 floats")
    h = handle or default_handle()
    check(lib().spmm_bsr32_analysis_f32(h.raw, direction, nnzb, _ptr(val), _ptr(masks),
                                        _ptr(val_col) if direction == DIRECTION_ROW else None),
          "spmm_bsr32_analysis_f32")
    return masks, (val_col if direction == DIRECTION_ROW else val)


def bsrmm_analysed(rowptr: torch.Tensor, colind: torch.Tensor, val_col: torch.Tensor,
                   masks: torch.Tensor, B: torch.Tensor, *, mb: int, kb: int, n: int, ldb: int,
                   order_b: int = ORDER_ROW, C: torch.Tensor, ldc: int,
                   order_c: int = ORDER_ROW, alpha: float = 1.0, beta: float = 0.0,
                   handle: Handle | None = None) -> torch.Tensor:
    """C(mb*32 x n) = alpha * A * B + beta * C on bsr32_analysis's output
    (spmm_bsrmm_analysed_f32)."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val_col, torch.float32, "val_col"), (masks, torch.int32, "masks"),
                      (B, torch.float32, "B"), (C, torch.float32, "C")):
        _need(t, dt, nm)
    nnzb = colind.numel()
    if val_col.numel() < nnzb * 1024 or masks.numel() < nnzb:
        raise ValueError("val_col / masks are shorter than the matrix's nnzb blocks")
    h = handle or default_handle()
    check(lib().spmm_bsrmm_analysed_f32(h.raw, mb, kb, n, nnzb, alpha, _ptr(rowptr),
                                        _ptr(colind), _ptr(val_col), _ptr(masks), _ptr(B), ldb,
                                        order_b, beta, _ptr(C), ldc, order_c),
          "spmm_bsrmm_analysed_f32")
    return C


def bsr16_analysis(val: torch.Tensor, *, nnzb: int, direction: int = DIRECTION_ROW,
                   masks: torch.Tensor | None = None, val_col: torch.Tensor | None = None,
                   handle: Handle | None = None):
    """bs = 16 fp16 form of bsr32_analysis (spmm_bsr16_analysis_f16): masks
    (int32, bit c < 16) and, for ROW blocks, the column-major fp16 copy."""
    _need(val, torch.float16, "val")
    if val.numel() < nnzb * 256:
        raise ValueError(f"val holds {val.numel()} halves, {nnzb} blocks need {nnzb * 256}")
    if masks is None:
        masks = torch.empty(max(nnzb, 1), dtype=torch.int32, device=val.device)
    if direction == DIRECTION_ROW and val_col is None:
        val_col = torch.empty(max(nnzb, 1) * 256, dtype=torch.float16, device=val.device)
    _need(masks, torch.int32, "masks")
    if masks.numel() < nnzb:
        raise ValueError("masks holds fewer than nnzb words")
    if direction == DIRECTION_ROW:
        _need(val_col, torch.float16, "val_col")
        if val_col.numel() < nnzb * 256:
            raise ValueError("val_col holds fewer than nnzb * 256 halves")
    h = handle or default_handle()
    check(lib().spmm_bsr16_analysis_f16(h.raw, direction, nnzb, _ptr(val), _ptr(masks),
                                        _ptr(val_col) if direction == DIRECTION_ROW else None),
          "spmm_bsr16_analysis_f16")
    return masks, (val_col if direction == DIRECTION_ROW else val)


def bsrmm_analysed_f16(rowptr: torch.Tensor, colind: torch.Tensor, val_col: torch.Tensor,
                       masks: torch.Tensor, B: torch.Tensor, *, mb: int, kb: int, n: int,
                       ldb: int, order_b: int = ORDER_ROW, C: torch.Tensor, ldc: int,
                       order_c: int = ORDER_ROW, alpha: float = 1.0, beta: float = 0.0,
                       handle: Handle | None = None) -> torch.Tensor:
    """fp16 A and B, fp32 C, on bsr16_analysis's output (spmm_bsrmm_analysed_f16)."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val_col, torch.float16, "val_col"), (masks, torch.int32, "masks"),
                      (B, torch.float16, "B"), (C, torch.float32, "C")):
        _need(t, dt, nm)
    nnzb = colind.numel()
    if val_col.numel() < nnzb * 256 or masks.numel() < nnzb:
        raise ValueError("val_col / masks are shorter than the matrix's nnzb blocks")
    h = handle or default_handle()
    check(lib().spmm_bsrmm_analysed_f16(h.raw, mb, kb, n, nnzb, alpha, _ptr(rowptr),
                                        _ptr(colind), _ptr(val_col), _ptr(masks), _ptr(B), ldb,
                                        order_b, beta, _ptr(C), ldc, order_c),
          "spmm_bsrmm_analysed_f16")
    return C


class _Grouped:
    """The analysis buffer of a grouped stream (a torch uint8 tensor owned by
    this object) and the plan the handle keeps for it: released by close(),
    by leaving a `with` block, or when the object is collected (a plan keyed
    by a freed address would otherwise outlive its buffer)."""

    BS, VT, ANALYSIS, PRODUCT, RELEASE = 0, None, "", "", ""

    def __init__(self, rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, *,
                 mb: int, group_rows: int, direction: int = DIRECTION_ROW,
                 handle: Handle | None = None):
        from ctypes import c_size_t
        self.buffer = None
        for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                          (val, self.VT, "val")):
            _need(t, dt, nm)
        nnzb = colind.numel()
        if mb < 0 or rowptr.numel() < mb + 1:
            raise ValueError(f"{type(self).__name__}: rowptr has {rowptr.numel()} entries, "
                             f"needs mb + 1 = {mb + 1}")
        if val.numel() < nnzb * self.BS * self.BS:
            raise ValueError(f"{type(self).__name__}: val has {val.numel()} entries, needs "
                             f"nnzb * {self.BS * self.BS} = {nnzb * self.BS * self.BS}")
        self.h = handle or default_handle()
        self.mb = mb
        size = c_size_t(0)
        args = (self.h.raw, direction, mb, nnzb, group_rows, _ptr(rowptr), _ptr(colind), _ptr(val))
        fn = getattr(lib(), self.ANALYSIS)
        check(fn(*args, None, byref(size)), self.ANALYSIS)
        buf = torch.empty(max(size.value, 1), dtype=torch.uint8, device=val.device)
        check(fn(*args, _ptr(buf), byref(size)), self.ANALYSIS)
        self.buffer = buf
        self.bytes = size.value
        # block rows per group: the header's word 0 (the library's choice when group_rows = 0)
        self.W = int(buf[:4].view(torch.int32).item()) if size.value >= 4 else group_rows
        # items: the last item pointer (item_ptr[ngroups] at byte 256 + 4 ngroups)
        ng = -(-mb // self.W) if self.W > 0 else 0
        off = 256 + 4 * ng
        self.nitems = (int(buf[off:off + 4].view(torch.int32).item())
                       if size.value >= off + 4 else 0)

    def mm(self, B: torch.Tensor, *, kb: int, n: int, ldb: int, C: torch.Tensor, ldc: int,
           order_b: int = ORDER_ROW, order_c: int = ORDER_ROW, alpha: float = 1.0,
           beta: float = 0.0) -> torch.Tensor:
        if self.buffer is None:
            raise ValueError(f"{type(self).__name__}: closed")
        _need(B, self.VT, "B")
        _need(C, torch.float32, "C")
        check(getattr(lib(), self.PRODUCT)(self.h.raw, self.mb, kb, n, _ptr(self.buffer), alpha,
                                           _ptr(B), ldb, order_b, beta, _ptr(C), ldc, order_c),
              self.PRODUCT)
        return C

    def close(self) -> None:
        if getattr(self, "buffer", None) is not None:
            getattr(lib(), self.RELEASE)(self.h.raw, _ptr(self.buffer))
            self.buffer = None

    def __enter__(self):
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GroupedBsr16(_Grouped):
    """spmm_bsr16_group_analysis_f16 on a bs = 16 fp16 BSR matrix (once), then
    .mm(...) = spmm_bsrmm_grouped_f16: the grouped stream, groups of
    group_rows adjacent block rows sharing their B-row copies (0: the library
    picks 2, 4 or 8 per matrix; .W holds the choice)."""

    BS, VT = 16, torch.float16
    ANALYSIS, PRODUCT = "spmm_bsr16_group_analysis_f16", "spmm_bsrmm_grouped_f16"
    RELEASE = "spmm_bsr16_group_release"

    def __init__(self, rowptr, colind, val, *, mb: int, group_rows: int = 0,
                 direction: int = DIRECTION_ROW, handle: Handle | None = None):
        super().__init__(rowptr, colind, val, mb=mb, group_rows=group_rows, direction=direction,
                         handle=handle)


class GroupedBsr32(_Grouped):
    """spmm_bsr32_group_analysis_f32 on a bs = 32 fp32 BSR matrix (once), then
    .mm(...) = spmm_bsrmm_grouped_f32: groups of group_rows (2 or 4) adjacent
    block rows sharing their B-row copies, each multiplying only its own
    nonzero columns (C bit-identical to bsrmm / bsrmm_analysed)."""

    BS, VT = 32, torch.float32
    ANALYSIS, PRODUCT = "spmm_bsr32_group_analysis_f32", "spmm_bsrmm_grouped_f32"
    RELEASE = "spmm_bsr_group_release"

    def __init__(self, rowptr, colind, val, *, mb: int, group_rows: int = 2,
                 direction: int = DIRECTION_ROW, handle: Handle | None = None):
        super().__init__(rowptr, colind, val, mb=mb, group_rows=group_rows, direction=direction,
                         handle=handle)


def bsrmm_f16(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, B: torch.Tensor, *,
              mb: int, kb: int, n: int, bs: int, ldb: int, order_b: int = ORDER_ROW,
              C: torch.Tensor, ldc: int, order_c: int = ORDER_ROW, alpha: float = 1.0,
              beta: float = 0.0, direction: int = DIRECTION_ROW,
              handle: Handle | None = None) -> torch.Tensor:
    """fp16 A and B, fp32 accumulate / C (spmm_bsrmm_ex_f16)."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val, torch.float16, "val"), (B, torch.float16, "B"),
                      (C, torch.float32, "C")):
        _need(t, dt, nm)
    h = handle or default_handle()
    check(lib().spmm_bsrmm_ex_f16(h.raw, direction, mb, kb, n, colind.numel(), bs, alpha,
                                  _ptr(rowptr), _ptr(colind), _ptr(val), _ptr(B), ldb, order_b,
                                  beta, _ptr(C), ldc, order_c), "spmm_bsrmm_ex_f16")
    return C


def hybrid_csrmm(csr: tuple, bsr: tuple, B: torch.Tensor, *, m: int, n: int, k: int, bs: int,
                 ldb: int, C: torch.Tensor, ldc: int, alpha: float = 1.0, beta: float = 0.0,
                 order_b: int = ORDER_ROW, order_c: int = ORDER_ROW,
                 handle: Handle | None = None) -> torch.Tensor:
    """Dense-block + CSR-remainder SpMM (divide.cu:348-373) on one stream:
    csr = (rowptr, colind, val), bsr = (rowptr, colind, val) from
    prep.divide. Row-major B and C (padded to whole blocks when the BSR part
    is non-empty): spmm_hybrid_csrmm_f32; other storage orders (divide.cu's
    column-major z, transB = N / T): spmm_hybrid_csrmm_ex_f32."""
    crp, cci, cv = csr
    brp, bci, bv = bsr
    for t, dt, nm in ((crp, torch.int32, "csr_rowptr"), (cci, torch.int32, "csr_colind"),
                      (cv, torch.float32, "csr_val"), (brp, torch.int32, "bsr_rowptr"),
                      (bci, torch.int32, "bsr_colind"), (bv, torch.float32, "bsr_val"),
                      (B, torch.float32, "B"), (C, torch.float32, "C")):
        _need(t, dt, nm)
    h = handle or default_handle()
    if order_b == ORDER_ROW and order_c == ORDER_ROW:
        check(lib().spmm_hybrid_csrmm_f32(h.raw, m, n, k, alpha, _ptr(crp), _ptr(cci), _ptr(cv),
                                          cci.numel(), bs, _ptr(brp), _ptr(bci), _ptr(bv),
                                          bci.numel(), _ptr(B), ldb, beta, _ptr(C), ldc),
              "spmm_hybrid_csrmm_f32")
    else:
        check(lib().spmm_hybrid_csrmm_ex_f32(h.raw, m, n, k, alpha, _ptr(crp), _ptr(cci),
                                             _ptr(cv), cci.numel(), bs, _ptr(brp), _ptr(bci),
                                             _ptr(bv), bci.numel(), _ptr(B), ldb, order_b, beta,
                                             _ptr(C), ldc, order_c), "spmm_hybrid_csrmm_ex_f32")
    return C


class _Descr:
    """spmm_mat_descr_t with an index base (cusparseMatDescr_t)."""

    def __init__(self, base: int = 0):
        self.raw = c_void_p()
        check(lib().spmm_create_mat_descr(byref(self.raw)), "spmm_create_mat_descr")
        check(lib().spmm_set_mat_index_base(self.raw, base), "spmm_set_mat_index_base")

    def __del__(self):
        try:
            lib().spmm_destroy_mat_descr(self.raw)
        except Exception:
            pass


def csr2bsr(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, *, m: int, n: int,
            bs: int, direction: int = DIRECTION_ROW, base: int = 0,
            handle: Handle | None = None):
    """Device csr2bsr (cusparseXcsr2bsrNnz + cusparseScsr2bsr semantics, rows
    sorted by column, bs <= 64) -> (bsr_rowptr, bsr_colind, bsr_val) tensors,
    index base `base` on both sides."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val, torch.float32, "val")):
        _need(t, dt, nm)
    h = handle or default_handle()
    da, dc = _Descr(base), _Descr(base)
    mb = (m + bs - 1) // bs
    brp = torch.empty(mb + 1, dtype=torch.int32, device=rowptr.device)
    nnzb = c_int(0)
    check(lib().spmm_xcsr2bsr_nnz_dev(h.raw, direction, m, n, da.raw, _ptr(rowptr), _ptr(colind),
                                      bs, dc.raw, _ptr(brp), byref(nnzb)),
          "spmm_xcsr2bsr_nnz_dev")
    bci = torch.empty(nnzb.value, dtype=torch.int32, device=rowptr.device)
    bval = torch.empty(nnzb.value * bs * bs, dtype=torch.float32, device=rowptr.device)
    if nnzb.value:
        check(lib().spmm_scsr2bsr_dev(h.raw, direction, m, n, da.raw, _ptr(val), _ptr(rowptr),
                                      _ptr(colind), bs, dc.raw, _ptr(bval), _ptr(brp),
                                      _ptr(bci)), "spmm_scsr2bsr_dev")
    return brp, bci, bval


def bsr_reblock32(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, *, mb: int,
                  bs: int, direction: int = DIRECTION_ROW, handle: Handle | None = None):
    """The same BSR matrix in 32 x 32 blocks (spmm_xbsr_reblock32_nnzb +
    spmm_sbsr_reblock32): a bs = 2 / 4 / 8 / 16 matrix onto the bs 32 MFMA streams.
    Returns (rowptr32, colind32, val32) with ceil(mb * bs / 32) block rows."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val, torch.float32, "val")):
        _need(t, dt, nm)
    nnzb = colind.numel()
    if rowptr.numel() < mb + 1 or val.numel() < nnzb * bs * bs:
        raise ValueError("bsr_reblock32: rowptr needs mb + 1 entries, val nnzb * bs^2")
    h = handle or default_handle()
    R = 32 // bs if bs in (2, 4, 8, 16, 32) else 0
    if not R:
        raise ValueError("bsr_reblock32: bs must divide 32")
    mb32 = (mb + R - 1) // R
    rp32 = torch.empty(mb32 + 1, dtype=torch.int32, device=val.device)
    nnzb32 = c_int(0)
    check(lib().spmm_xbsr_reblock32_nnzb(h.raw, direction, mb, nnzb, bs, _ptr(rowptr),
                                         _ptr(colind), _ptr(rp32), byref(nnzb32)),
          "spmm_xbsr_reblock32_nnzb")
    ci32 = torch.empty(max(nnzb32.value, 1), dtype=torch.int32, device=val.device)
    v32 = torch.empty(max(nnzb32.value, 1) * 1024, dtype=torch.float32, device=val.device)
    check(lib().spmm_sbsr_reblock32(h.raw, direction, mb, nnzb, bs, _ptr(rowptr), _ptr(colind),
                                    _ptr(val), _ptr(rp32), nnzb32.value, _ptr(ci32), _ptr(v32)),
          "spmm_sbsr_reblock32")
    return rp32, ci32[:nnzb32.value], v32[:nnzb32.value * 1024]


def bsr2csr(rowptr: torch.Tensor, colind: torch.Tensor, val: torch.Tensor, *, mb: int, nb: int,
            bs: int, direction: int = DIRECTION_ROW, base: int = 0,
            handle: Handle | None = None):
    """Device bsr2csr (cusparseSbsr2csr semantics: every block expanded,
    nnz = nnzb * bs^2) -> (csr_rowptr, csr_colind, csr_val) tensors."""
    for t, dt, nm in ((rowptr, torch.int32, "rowptr"), (colind, torch.int32, "colind"),
                      (val, torch.float32, "val")):
        _need(t, dt, nm)
    h = handle or default_handle()
    da, dc = _Descr(base), _Descr(base)
    nnz = colind.numel() * bs * bs
    crp = torch.empty(mb * bs + 1, dtype=torch.int32, device=rowptr.device)
    cci = torch.empty(nnz, dtype=torch.int32, device=rowptr.device)
    cv = torch.empty(nnz, dtype=torch.float32, device=rowptr.device)
    check(lib().spmm_sbsr2csr_dev(h.raw, direction, mb, nb, da.raw, _ptr(val), _ptr(rowptr),
                                  _ptr(colind), bs, dc.raw, _ptr(cv), _ptr(crp), _ptr(cci)),
          "spmm_sbsr2csr_dev")
    return crp, cci, cv


def coo2csr(coo_row: torch.Tensor, m: int, base: int = 0,
            handle: Handle | None = None) -> torch.Tensor:
    """cusparseXcoo2csr (csrmm.cu:148-149): int32[m+1] row pointer of a
    row-sorted COO whose row indices are in `base`."""
    _need(coo_row, torch.int32, "coo_row")
    h = handle or default_handle()
    rp = torch.empty(m + 1, dtype=torch.int32, device=coo_row.device)
    check(lib().spmm_xcoo2csr(h.raw, _ptr(coo_row), coo_row.numel(), m, _ptr(rp), base),
          "spmm_xcoo2csr")
    return rp


class MultiGPU:
    """spmm_multi_t (include/spmm_multi.h): one host thread drives the row
    shards of a CSR x dense product on several GPUs, RCCL communicators from
    ncclCommInitAll; every device's rows go straight into the same rows of
    every device's m x n C (grouped ncclSend / ncclRecv of exact shards)."""

    def __init__(self, devices: list[int]):
        self._c = c_void_p()
        arr = (c_int * len(devices))(*devices)
        check(lib().spmm_multi_create(byref(self._c), len(devices), arr), "spmm_multi_create")
        self.devices = list(devices)

    @staticmethod
    def slot_rows(bounds, chunks: int = 1) -> int:
        """Rows per chunk (spmm_multi_slot_rows)."""
        b = (c_int * len(bounds))(*[int(x) for x in bounds])
        return lib().spmm_multi_slot_rows(len(bounds) - 1, b, chunks)

    def csrmm(self, bounds, parts, part_nnz, Bs, Cs, *, m: int, n: int, k: int, ldb: int,
              ldc: int, chunks: int = 1) -> None:
        """parts[p] = (rowptr, colind, val) tensors on device p (rowptr of the
        part's rows, indexing colind / val directly); Bs[p] B replicas; Cs[p]
        the m x n row-major outputs with leading dimension ldc, one per device,
        each complete after the call (include/spmm_multi.h).
        Ordered against each device's current torch stream: the kernels start
        after the work already queued there, and work queued there afterwards
        sees all of C (spmm_multi_set_user_streams)."""
        P = len(self.devices)
        if not (len(parts) == len(part_nnz) == len(Bs) == len(Cs) == P) or len(bounds) != P + 1:
            raise ValueError(f"MultiGPU.csrmm: {P} parts expected")
        if chunks < 1 or ldc < n or ldb < n:
            raise ValueError("MultiGPU.csrmm: chunks >= 1, ldb >= n and ldc >= n")
        if int(bounds[0]) != 0 or int(bounds[-1]) != m:
            raise ValueError(f"MultiGPU.csrmm: bounds must run from 0 to m = {m}")
        need_c = (m - 1) * ldc + n if m > 0 else 0
        for p in range(P):
            rp, ci, v = parts[p]
            for t, dt, nm in ((rp, torch.int32, "rowptr"), (ci, torch.int32, "colind"),
                              (v, torch.float32, "val"), (Bs[p], torch.float32, "B"),
                              (Cs[p], torch.float32, "C")):
                _need(t, dt, nm)
                if t.device.index != self.devices[p]:
                    raise ValueError(f"part {p}: {nm} is on {t.device}, expected "
                                     f"cuda:{self.devices[p]}")
            rows = int(bounds[p + 1]) - int(bounds[p])
            if rp.numel() < rows + 1:
                raise ValueError(f"part {p}: rowptr has {rp.numel()} entries, needs {rows + 1}")
            if Cs[p].numel() < need_c:
                raise ValueError(f"part {p}: C has {Cs[p].numel()} floats, the m x n output "
                                 f"with ldc {ldc} needs {need_c}")
            if k > 0 and Bs[p].numel() < (k - 1) * ldb + n:
                raise ValueError(f"part {p}: B has {Bs[p].numel()} floats, needs "
                                 f"{(k - 1) * ldb + n}")
        vp = lambda ts: (c_void_p * P)(*[_ptr(t) for t in ts])  # noqa: E731
        streams = (c_void_p * P)(*[torch.cuda.current_stream(d).cuda_stream
                                   for d in self.devices])
        check(lib().spmm_multi_set_user_streams(self._c, streams),
              "spmm_multi_set_user_streams")
        b = (c_int * (P + 1))(*[int(x) for x in bounds])
        nz = (c_int * P)(*[int(x) for x in part_nnz])
        check(lib().spmm_csr_f32_multi(self._c, m, n, k, b, vp([q[0] for q in parts]),
                                       vp([q[1] for q in parts]), vp([q[2] for q in parts]), nz,
                                       vp(Bs), ldb, vp(Cs), ldc, chunks), "spmm_csr_f32_multi")

    def synchronize(self) -> None:
        check(lib().spmm_multi_synchronize(self._c), "spmm_multi_synchronize")

    def set_timing(self, enable: bool) -> None:
        check(lib().spmm_multi_set_timing(self._c, int(enable)), "spmm_multi_set_timing")

    def times(self) -> tuple[list[float], list[float]]:
        """(compute_ms, total_ms) per part of the last call."""
        P = len(self.devices)
        a, t = (c_float * P)(), (c_float * P)()
        check(lib().spmm_multi_get_times(self._c, a, t), "spmm_multi_get_times")
        return list(a), list(t)

    def close(self) -> None:
        if getattr(self, "_c", None) is not None and self._c.value:
            lib().spmm_multi_destroy(self._c)
            self._c = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["coo2csr", "MultiGPU", "csr2bsr", "bsr2csr", "Handle", "hybrid_csrmm", "default_handle", "gespmm_csrmm", "csrmm", "bsrmm", "bsrmm_f16",
           "SpmmError", "ORDER_ROW", "ORDER_COL"]
