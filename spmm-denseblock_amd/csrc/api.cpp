// api.cpp — extern "C" SpMM entry points: argument checks (mirroring the
// reference's status behaviour) and dispatch to the HIP launchers.
#include <cstdint>
#include <cstdlib>

#include "context.hpp"

using namespace spmm;

namespace {

// Workspace carve-up: [carries | staged B | staged C], 256-byte aligned.
struct WsLayout {
  size_t carry_off = 0, carry_bytes = 0, b_off = 0, c_off = 0, total = 0;
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

spmm_status_t csrmm_impl(spmm_context* ctx, int m, int n, int k, int nnz_hint, float alpha,
                         const int* rowptr, const int* colind, const float* val, int base,
                         const float* B, int ldb, spmm_order_t orderB, float beta, float* C,
                         int ldc, spmm_order_t orderC, bool hot = false) {
  WsLayout L;
  L.carry_bytes = csrmm_carry_bytes(ctx, m, n);
  L.b_off = align256(L.carry_bytes);
  const size_t b_bytes = orderB == SPMM_ORDER_COL ? (size_t)k * n * sizeof(float) : 0;
  L.c_off = align256(L.b_off + b_bytes);
  const size_t c_bytes = orderC == SPMM_ORDER_COL ? (size_t)m * n * sizeof(float) : 0;
  L.total = L.c_off + c_bytes;
  spmm_status_t st = ensure_workspace(ctx, L.total);
  if (st != SPMM_STATUS_SUCCESS) return st;
  char* ws = static_cast<char*>(ctx->ws);

  const float* Bx = B;
  int ldbx = ldb;
  // hot-tagged indices: one buffer resource for all of B when every row offset
  // fits 32 bits (the kernel then passes the row in soffset)
  auto hot_mode = [&](int ld) {
    return !hot ? 0 : ((long long)(k + base) * ld + n) * 4 + 64 < (1ll << 32) ? 2 : 1;
  };
  if (orderB == SPMM_ORDER_COL) {
    // B (k x n col-major) is an (n x k) row-major matrix with ld ldb.
    float* Bt = reinterpret_cast<float*>(ws + L.b_off);
    st = launch_transpose(ctx, n, k, B, ldb, Bt, n, 0.f);
    if (st != SPMM_STATUS_SUCCESS) return st;
    Bx = Bt;
    ldbx = n;
  }
  if (orderC == SPMM_ORDER_ROW) {
    return launch_csrmm_rowmajor(ctx, m, n, rowptr, colind, val, base, Bx, ldbx, alpha, beta, C,
                                 ldc, ws, nnz_hint, hot_mode(ldbx));
  }
  float* Ct = reinterpret_cast<float*>(ws + L.c_off);
  st = launch_csrmm_rowmajor(ctx, m, n, rowptr, colind, val, base, Bx, ldbx, alpha, 0.f, Ct, n,
                             ws, nnz_hint, hot_mode(ldbx));
  if (st != SPMM_STATUS_SUCCESS) return st;
  // C (m x n col-major, ldc) is an (n x m) row-major matrix with ld ldc.
  return launch_transpose(ctx, m, n, Ct, n, C, ldc, beta);
}

// Column-major B and / or C with ROW blocks at bs 16 / 32 / 64 and 2 / 4 / 8
// fp32 (cusparseSbsrmm's transB = N layout, run_bsrmm.cu:70-71) run on the
// row-major-B kernels (column streams, column-masked LDS kernels, the
// lane-group kernel)
// (DESIGN.md §4): B is transposed into a row-major workspace copy (the kernels
// copy whole B-panel rows), C is written column-major by the kernels' own
// LDS-transposed epilogue. The direct kernels for these layouts fetch B
// fragment-wise and were 2.6x (bs 32) to 4.5x (bs 16 fp16) slower end to end.
// Any other shape keeps the direct kernels.
bool bsr_stage(spmm_direction_t dir, int bs, int n, int elem, spmm_order_t ob, spmm_order_t oc,
               const void* val) {
  const int vec = 16 / elem;  // elements per 16-byte copy
  const bool f32_stream = elem == 4 && (bs == 2 || bs == 4 || bs == 8 || bs == 32 || bs == 64);
  return dir == SPMM_DIRECTION_ROW && (bs == 16 || f32_stream) &&
         (ob == SPMM_ORDER_COL || oc == SPMM_ORDER_COL) && n >= vec && n % vec == 0 &&
         reinterpret_cast<uintptr_t>(val) % 16 == 0;
}

template <typename T, typename Launch>
spmm_status_t bsrmm_staged(spmm_context* ctx, int kb, int n, int bs, const T* B, int ldb,
                           spmm_order_t ob, Launch&& launch) {
  if (ob == SPMM_ORDER_ROW) return launch(B, ldb);
  spmm_status_t st = ensure_workspace(ctx, (size_t)kb * bs * n * sizeof(T));
  if (st != SPMM_STATUS_SUCCESS) return st;
  // B (kb*bs x n col-major) is an (n x kb*bs) row-major matrix with ld ldb.
  T* Bt = static_cast<T*>(ctx->ws);
  if constexpr (sizeof(T) == 4)
    st = launch_transpose(ctx, n, kb * bs, B, ldb, Bt, n, 0.f);
  else
    st = launch_transpose16(ctx, n, kb * bs, B, ldb, Bt, n);
  if (st != SPMM_STATUS_SUCCESS) return st;
  return launch(Bt, n);
}

// [a, a + bytes) and [b, b + bytes) share a byte
bool overlaps(const void* a, const void* b, size_t bytes) {
  const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
  return x < y + bytes && y < x + bytes;
}

}  // namespace

extern "C" {

spmm_status_t spmm_gespmm_csrmm_f32(int A_nrows, int B_ncols, const int* A_rowPtr,
                                    const int* A_colInd, const float* A_val, const float* B,
                                    float* C, void* stream) {
  if (A_nrows < 0 || B_ncols < 0) return SPMM_STATUS_INVALID_VALUE;
  if (A_nrows == 0 || B_ncols == 0) return SPMM_STATUS_SUCCESS;
  if (!A_rowPtr || !A_colInd || !A_val || !B || !C) return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = default_context();
  if (!ctx) return SPMM_STATUS_NOT_INITIALIZED;
  ctx->stream = reinterpret_cast<hipStream_t>(stream);
  // nnz is only known on the device (A_rowPtr[A_nrows]); -1 sizes the grid
  // from the row count.
  return csrmm_impl(ctx, A_nrows, B_ncols, A_nrows, -1, 1.f, A_rowPtr, A_colInd, A_val, 0, B,
                    B_ncols, SPMM_ORDER_ROW, 0.f, C, B_ncols, SPMM_ORDER_ROW);
}

spmm_status_t spmm_csrmm_ex_f32(spmm_handle_t handle, int m, int n, int k, int nnz, float alpha,
                                const int* csrRowPtr, const int* csrColInd, const float* csrVal,
                                spmm_index_base_t base, const float* B, int ldb,
                                spmm_order_t orderB, float beta, float* C, int ldc,
                                spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (m < 0 || n < 0 || k < 0 || nnz < 0) return SPMM_STATUS_INVALID_VALUE;
  if (base != SPMM_INDEX_BASE_ZERO && base != SPMM_INDEX_BASE_ONE)
    return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!csrRowPtr || !C || (k > 0 && !B) || (nnz > 0 && (!csrColInd || !csrVal)))
    return SPMM_STATUS_INVALID_VALUE;
  if (orderB == SPMM_ORDER_ROW ? ldb < n : ldb < (k > 0 ? k : 1)) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_ROW ? ldc < n : ldc < m) return SPMM_STATUS_INVALID_VALUE;
  return csrmm_impl(handle, m, n, k, nnz, alpha, csrRowPtr, csrColInd, csrVal, (int)base, B, ldb,
                    orderB, beta, C, ldc, orderC);
}

spmm_status_t spmm_csr_hot_analysis(spmm_handle_t handle, int n, int k, int nnz,
                                    const int* csrColInd, spmm_index_base_t base,
                                    long long hotBytes, int* csrColIndHot) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (n < 0 || k < 0 || nnz < 0 || hotBytes < 0) return SPMM_STATUS_INVALID_VALUE;
  if (base != SPMM_INDEX_BASE_ZERO && base != SPMM_INDEX_BASE_ONE)
    return SPMM_STATUS_INVALID_VALUE;
  if (nnz == 0) return SPMM_STATUS_SUCCESS;
  if (!csrColInd || !csrColIndHot || k == 0) return SPMM_STATUS_INVALID_VALUE;
  // one gathered B-row piece: the merge-path kernel's column tile (64 / 128 / 256
  // floats) or the whole row when n is narrower
  const long long tile = n > 128 ? 256 : (n > 64 ? 128 : 64);
  const long long piece = 4 * (n > 0 && n < tile ? n : tile);
  const long long hot_rows = (hotBytes ? hotBytes : SPMM_CSR_HOT_BYTES_DEFAULT) / piece;
  return launch_csr_hot_analysis(handle, k, nnz, csrColInd, (int)base, hot_rows, csrColIndHot);
}

spmm_status_t spmm_csrmm_hot_f32(spmm_handle_t handle, int m, int n, int k, int nnz, float alpha,
                                 const int* csrRowPtr, const int* csrColIndHot,
                                 const float* csrVal, spmm_index_base_t base, const float* B,
                                 int ldb, spmm_order_t orderB, float beta, float* C, int ldc,
                                 spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (m < 0 || n < 0 || k < 0 || nnz < 0) return SPMM_STATUS_INVALID_VALUE;
  if (base != SPMM_INDEX_BASE_ZERO && base != SPMM_INDEX_BASE_ONE)
    return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!csrRowPtr || !C || (k > 0 && !B) || (nnz > 0 && (!csrColIndHot || !csrVal)))
    return SPMM_STATUS_INVALID_VALUE;
  if (orderB == SPMM_ORDER_ROW ? ldb < n : ldb < (k > 0 ? k : 1)) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_ROW ? ldc < n : ldc < m) return SPMM_STATUS_INVALID_VALUE;
  return csrmm_impl(handle, m, n, k, nnz, alpha, csrRowPtr, csrColIndHot, csrVal, (int)base, B,
                    ldb, orderB, beta, C, ldc, orderC, true);
}

spmm_status_t spmm_scsrmm2(spmm_handle_t handle, spmm_operation_t transA,
                           spmm_operation_t transB, int m, int n, int k, int nnz,
                           const float* alpha, const spmm_mat_descr_t descrA,
                           const float* csrValA, const int* csrRowPtrA, const int* csrColIndA,
                           const float* B, int ldb, const float* beta, float* C, int ldc) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (!descrA || !alpha || !beta) return SPMM_STATUS_INVALID_VALUE;
  if (transA != SPMM_OPERATION_NON_TRANSPOSE) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (transB != SPMM_OPERATION_NON_TRANSPOSE && transB != SPMM_OPERATION_TRANSPOSE)
    return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  const spmm_order_t ob =
      transB == SPMM_OPERATION_NON_TRANSPOSE ? SPMM_ORDER_COL : SPMM_ORDER_ROW;
  return spmm_csrmm_ex_f32(handle, m, n, k, nnz, *alpha, csrRowPtrA, csrColIndA, csrValA,
                           descrA->base, B, ldb, ob, *beta, C, ldc, SPMM_ORDER_COL);
}

spmm_status_t spmm_scsrmm(spmm_handle_t handle, spmm_operation_t transA, int m, int n, int k,
                          int nnz, const float* alpha, const spmm_mat_descr_t descrA,
                          const float* csrValA, const int* csrRowPtrA, const int* csrColIndA,
                          const float* B, int ldb, const float* beta, float* C, int ldc) {
  return spmm_scsrmm2(handle, transA, SPMM_OPERATION_NON_TRANSPOSE, m, n, k, nnz, alpha, descrA,
                      csrValA, csrRowPtrA, csrColIndA, B, ldb, beta, C, ldc);
}

static spmm_status_t bsr_checks(int mb, int kb, int n, int nnzb, int bs, const int* rowptr,
                                const int* colind, const void* val, const void* B, int ldb,
                                spmm_order_t orderB, const void* C, int ldc,
                                spmm_order_t orderC, bool* quick) {
  *quick = false;
  if (mb < 0 || n < 0 || kb < 0 || nnzb < 0 || bs <= 0) return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  // Quick return (rocsparse_bsrmm.h:152-154): C is left untouched.
  if (mb == 0 || n == 0 || kb == 0 || nnzb == 0) {
    *quick = true;
    return SPMM_STATUS_SUCCESS;
  }
  if (!val || !rowptr || !colind || !B || !C) return SPMM_STATUS_INVALID_VALUE;
  const long long K = (long long)kb * bs, M = (long long)mb * bs;
  if (orderB == SPMM_ORDER_COL ? ldb < K : ldb < n) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_COL ? ldc < M : ldc < n) return SPMM_STATUS_INVALID_VALUE;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_bsrmm_ex_f32(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb, int n,
                                int nnzb, int blockDim, float alpha, const int* bsrRowPtr,
                                const int* bsrColInd, const float* bsrVal, const float* B, int ldb,
                                spmm_order_t orderB, float beta, float* C, int ldc,
                                spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  bool quick = false;
  spmm_status_t st = bsr_checks(mb, kb, n, nnzb, blockDim, bsrRowPtr, bsrColInd, bsrVal, B, ldb,
                                orderB, C, ldc, orderC, &quick);
  if (st != SPMM_STATUS_SUCCESS || quick) return st;
  if (bsr_stage(dir, blockDim, n, 4, orderB, orderC, bsrVal))
    return bsrmm_staged<float>(handle, kb, n, blockDim, B, ldb, orderB,
                               [&](const float* Bx, int ldbx) {
                                 return launch_bsrmm_f32(handle, dir, mb, kb, n, nnzb, blockDim,
                                                         alpha, bsrRowPtr, bsrColInd, bsrVal, Bx,
                                                         ldbx, SPMM_ORDER_ROW, beta, C, ldc,
                                                         orderC);
                               });
  return launch_bsrmm_f32(handle, dir, mb, kb, n, nnzb, blockDim, alpha, bsrRowPtr, bsrColInd,
                          bsrVal, B, ldb, orderB, beta, C, ldc, orderC);
}

spmm_status_t spmm_bsr32_analysis_f32(spmm_handle_t handle, spmm_direction_t dir, int nnzb,
                                      const float* bsrVal, unsigned* masks, float* valCol) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) || nnzb < 0)
    return SPMM_STATUS_INVALID_VALUE;
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  if (!bsrVal || !masks || (dir == SPMM_DIRECTION_ROW && !valCol))
    return SPMM_STATUS_INVALID_VALUE;
  if (reinterpret_cast<uintptr_t>(bsrVal) % 16 != 0) return SPMM_STATUS_INVALID_VALUE;
  if (dir == SPMM_DIRECTION_ROW && overlaps(bsrVal, valCol, (size_t)nnzb * 1024 * sizeof(float)))
    return SPMM_STATUS_INVALID_VALUE;
  return launch_bsr32_analysis(handle, dir, nnzb, bsrVal, masks, valCol);
}

spmm_status_t spmm_bsrmm_analysed_f32(spmm_handle_t handle, int mb, int kb, int n, int nnzb,
                                      float alpha, const int* bsrRowPtr, const int* bsrColInd,
                                      const float* valCol, const unsigned* masks, const float* B,
                                      int ldb, spmm_order_t orderB, float beta, float* C,
                                      int ldc, spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  bool quick = false;
  spmm_status_t st = bsr_checks(mb, kb, n, nnzb, 32, bsrRowPtr, bsrColInd, valCol, B, ldb,
                                orderB, C, ldc, orderC, &quick);
  if (st != SPMM_STATUS_SUCCESS || quick) return st;
  if (!masks) return SPMM_STATUS_INVALID_VALUE;
  const auto launch = [&](const float* Bx, int ldbx, spmm_order_t obx) {
    return launch_bsrmm_f32(handle, SPMM_DIRECTION_COLUMN, mb, kb, n, nnzb, 32, alpha, bsrRowPtr,
                            bsrColInd, valCol, Bx, ldbx, obx, beta, C, ldc, orderC, false, masks);
  };
  // a column-major B is staged row-major (the column stream copies whole B rows)
  if (orderB == SPMM_ORDER_COL && n >= 4 && n % 4 == 0)
    return bsrmm_staged<float>(handle, kb, n, 32, B, ldb, orderB,
                               [&](const float* Bx, int ldbx) {
                                 return launch(Bx, ldbx, SPMM_ORDER_ROW);
                               });
  return launch(B, ldb, orderB);
}

spmm_status_t spmm_bsr16_analysis_f16(spmm_handle_t handle, spmm_direction_t dir, int nnzb,
                                      const uint16_t* bsrVal, unsigned* masks, uint16_t* valCol) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) || nnzb < 0)
    return SPMM_STATUS_INVALID_VALUE;
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  if (!bsrVal || !masks || (dir == SPMM_DIRECTION_ROW && !valCol))
    return SPMM_STATUS_INVALID_VALUE;
  if (reinterpret_cast<uintptr_t>(bsrVal) % 8 != 0) return SPMM_STATUS_INVALID_VALUE;
  if (dir == SPMM_DIRECTION_ROW && overlaps(bsrVal, valCol, (size_t)nnzb * 256 * sizeof(uint16_t)))
    return SPMM_STATUS_INVALID_VALUE;
  return launch_bsr16_analysis(handle, dir, nnzb, bsrVal, masks, valCol);
}

spmm_status_t spmm_bsrmm_analysed_f16(spmm_handle_t handle, int mb, int kb, int n, int nnzb,
                                      float alpha, const int* bsrRowPtr, const int* bsrColInd,
                                      const uint16_t* valCol, const unsigned* masks,
                                      const uint16_t* B, int ldb, spmm_order_t orderB,
                                      float beta, float* C, int ldc, spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  bool quick = false;
  spmm_status_t st = bsr_checks(mb, kb, n, nnzb, 16, bsrRowPtr, bsrColInd, valCol, B, ldb,
                                orderB, C, ldc, orderC, &quick);
  if (st != SPMM_STATUS_SUCCESS || quick) return st;
  if (!masks) return SPMM_STATUS_INVALID_VALUE;
  const auto launch = [&](const uint16_t* Bx, int ldbx, spmm_order_t obx) {
    return launch_bsrmm_f16(handle, SPMM_DIRECTION_COLUMN, mb, kb, n, nnzb, 16, alpha, bsrRowPtr,
                            bsrColInd, valCol, Bx, ldbx, obx, beta, C, ldc, orderC, masks);
  };
  if (orderB == SPMM_ORDER_COL && n >= 128 && n % 8 == 0)
    return bsrmm_staged<uint16_t>(handle, kb, n, 16, B, ldb, orderB,
                                  [&](const uint16_t* Bx, int ldbx) {
                                    return launch(Bx, ldbx, SPMM_ORDER_ROW);
                                  });
  return launch(B, ldb, orderB);
}

spmm_status_t spmm_bsrmm_ex_f16(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb, int n,
                                int nnzb, int blockDim, float alpha, const int* bsrRowPtr,
                                const int* bsrColInd, const uint16_t* bsrVal, const uint16_t* B,
                                int ldb, spmm_order_t orderB, float beta, float* C, int ldc,
                                spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  bool quick = false;
  spmm_status_t st = bsr_checks(mb, kb, n, nnzb, blockDim, bsrRowPtr, bsrColInd, bsrVal, B, ldb,
                                orderB, C, ldc, orderC, &quick);
  if (st != SPMM_STATUS_SUCCESS || quick) return st;
  if (bsr_stage(dir, blockDim, n, 2, orderB, orderC, bsrVal))
    return bsrmm_staged<uint16_t>(handle, kb, n, blockDim, B, ldb, orderB,
                                  [&](const uint16_t* Bx, int ldbx) {
                                    return launch_bsrmm_f16(handle, dir, mb, kb, n, nnzb,
                                                            blockDim, alpha, bsrRowPtr, bsrColInd,
                                                            bsrVal, Bx, ldbx, SPMM_ORDER_ROW, beta,
                                                            C, ldc, orderC);
                                  });
  return launch_bsrmm_f16(handle, dir, mb, kb, n, nnzb, blockDim, alpha, bsrRowPtr, bsrColInd,
                          bsrVal, B, ldb, orderB, beta, C, ldc, orderC);
}

spmm_status_t spmm_csrmm_ex_f64(spmm_handle_t handle, int m, int n, int k, int nnz, double alpha,
                                const int* csrRowPtr, const int* csrColInd, const double* csrVal,
                                spmm_index_base_t base, const double* B, int ldb,
                                spmm_order_t orderB, double beta, double* C, int ldc,
                                spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (m < 0 || n < 0 || k < 0 || nnz < 0) return SPMM_STATUS_INVALID_VALUE;
  if (base != SPMM_INDEX_BASE_ZERO && base != SPMM_INDEX_BASE_ONE)
    return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!csrRowPtr || !C || (k > 0 && !B) || (nnz > 0 && (!csrColInd || !csrVal)))
    return SPMM_STATUS_INVALID_VALUE;
  if (orderB == SPMM_ORDER_ROW ? ldb < n : ldb < (k > 0 ? k : 1)) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_ROW ? ldc < n : ldc < m) return SPMM_STATUS_INVALID_VALUE;
  return launch_csrmm_f64(handle, m, n, csrRowPtr, csrColInd, csrVal, (int)base, B, ldb,
                          orderB == SPMM_ORDER_ROW, alpha, beta, C, ldc, orderC == SPMM_ORDER_ROW);
}

spmm_status_t spmm_dcsrmm2(spmm_handle_t handle, spmm_operation_t transA,
                           spmm_operation_t transB, int m, int n, int k, int nnz,
                           const double* alpha, const spmm_mat_descr_t descrA,
                           const double* csrValA, const int* csrRowPtrA, const int* csrColIndA,
                           const double* B, int ldb, const double* beta, double* C, int ldc) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (!descrA || !alpha || !beta) return SPMM_STATUS_INVALID_VALUE;
  if (transA != SPMM_OPERATION_NON_TRANSPOSE) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (transB != SPMM_OPERATION_NON_TRANSPOSE && transB != SPMM_OPERATION_TRANSPOSE)
    return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  const spmm_order_t ob =
      transB == SPMM_OPERATION_NON_TRANSPOSE ? SPMM_ORDER_COL : SPMM_ORDER_ROW;
  return spmm_csrmm_ex_f64(handle, m, n, k, nnz, *alpha, csrRowPtrA, csrColIndA, csrValA,
                           descrA->base, B, ldb, ob, *beta, C, ldc, SPMM_ORDER_COL);
}

spmm_status_t spmm_gespmm_csrmm_f64(int A_nrows, int B_ncols, const int* A_rowPtr,
                                    const int* A_colInd, const double* A_val, const double* B,
                                    double* C, void* stream) {
  spmm_context* ctx = default_context();
  if (!ctx) return SPMM_STATUS_NOT_INITIALIZED;
  if (A_nrows < 0 || B_ncols < 0) return SPMM_STATUS_INVALID_VALUE;
  if (A_nrows == 0 || B_ncols == 0) return SPMM_STATUS_SUCCESS;
  if (!A_rowPtr || !C || !B) return SPMM_STATUS_INVALID_VALUE;
  hipStream_t saved = ctx->stream;
  ctx->stream = reinterpret_cast<hipStream_t>(stream);
  const spmm_status_t st = launch_csrmm_f64(ctx, A_nrows, B_ncols, A_rowPtr, A_colInd, A_val, 0,
                                            B, B_ncols, true, 1.0, 0.0, C, B_ncols, true);
  ctx->stream = saved;
  return st;
}

spmm_status_t spmm_bsrmm_ex_f64(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb, int n,
                                int nnzb, int blockDim, double alpha, const int* bsrRowPtr,
                                const int* bsrColInd, const double* bsrVal, const double* B,
                                int ldb, spmm_order_t orderB, double beta, double* C, int ldc,
                                spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  bool quick = false;
  spmm_status_t st = bsr_checks(mb, kb, n, nnzb, blockDim, bsrRowPtr, bsrColInd, bsrVal, B, ldb,
                                orderB, C, ldc, orderC, &quick);
  if (st != SPMM_STATUS_SUCCESS || quick) return st;
  return launch_bsrmm_f64(handle, dir, mb, n, blockDim, bsrRowPtr, bsrColInd, bsrVal, B, ldb,
                          orderB == SPMM_ORDER_ROW, alpha, beta, C, ldc, orderC == SPMM_ORDER_ROW);
}

spmm_status_t spmm_dbsrmm(spmm_handle_t handle, spmm_direction_t dir, spmm_operation_t transA,
                          spmm_operation_t transB, int mb, int n, int kb, int nnzb,
                          const double* alpha, const spmm_mat_descr_t descrA,
                          const double* bsrValA, const int* bsrRowPtrA, const int* bsrColIndA,
                          int blockDim, const double* B, int ldb, const double* beta, double* C,
                          int ldc) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (!descrA) return SPMM_STATUS_INVALID_VALUE;
  if (transA != SPMM_OPERATION_NON_TRANSPOSE) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (transB != SPMM_OPERATION_NON_TRANSPOSE && transB != SPMM_OPERATION_TRANSPOSE)
    return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (mb < 0 || n < 0 || kb < 0 || nnzb < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (mb == 0 || n == 0 || kb == 0 || nnzb == 0) return SPMM_STATUS_SUCCESS;
  if (!alpha || !beta) return SPMM_STATUS_INVALID_VALUE;
  if (descrA->base != SPMM_INDEX_BASE_ZERO) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  const spmm_order_t ob =
      transB == SPMM_OPERATION_NON_TRANSPOSE ? SPMM_ORDER_COL : SPMM_ORDER_ROW;
  return spmm_bsrmm_ex_f64(handle, dir, mb, kb, n, nnzb, blockDim, *alpha, bsrRowPtrA, bsrColIndA,
                           bsrValA, B, ldb, ob, *beta, C, ldc, SPMM_ORDER_COL);
}

spmm_status_t spmm_sbsrmm(spmm_handle_t handle, spmm_direction_t dir, spmm_operation_t transA,
                          spmm_operation_t transB, int mb, int n, int kb, int nnzb,
                          const float* alpha, const spmm_mat_descr_t descrA,
                          const float* bsrValA, const int* bsrRowPtrA, const int* bsrColIndA,
                          int blockDim, const float* B, int ldb, const float* beta, float* C,
                          int ldc) {
  // Check order follows rocsparse_bsrmm.h:109-176.
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (!descrA) return SPMM_STATUS_INVALID_VALUE;
  if (transA != SPMM_OPERATION_NON_TRANSPOSE) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (transB != SPMM_OPERATION_NON_TRANSPOSE && transB != SPMM_OPERATION_TRANSPOSE)
    return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  if (mb < 0 || n < 0 || kb < 0 || nnzb < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (mb == 0 || n == 0 || kb == 0 || nnzb == 0) return SPMM_STATUS_SUCCESS;
  if (!alpha || !beta) return SPMM_STATUS_INVALID_VALUE;
  if (descrA->base != SPMM_INDEX_BASE_ZERO) return SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED;
  const spmm_order_t ob =
      transB == SPMM_OPERATION_NON_TRANSPOSE ? SPMM_ORDER_COL : SPMM_ORDER_ROW;
  return spmm_bsrmm_ex_f32(handle, dir, mb, kb, n, nnzb, blockDim, *alpha, bsrRowPtrA, bsrColIndA,
                           bsrValA, B, ldb, ob, *beta, C, ldc, SPMM_ORDER_COL);
}

}  // extern "C"

// Mean CSR-remainder entries per 32-row block row up to which the hybrid runs
// fused by default (products stand-in 71: fused 2.02 vs 2.68 ms; reddit 222:
// 0.90 vs 0.96; RCM-reordered reddit 2295: 1.94 vs 2.02 since the fused kernel
// starts the longest block rows first, 2.04 vs 2.03 before;
// profiles/r02_hybrid_order_sweep.jsonl). Past it the merge-path CSR kernel's
// balance is kept.
constexpr int64_t kHybridFusedRemainderPerBlockRow = 4096;

extern "C" spmm_status_t spmm_hybrid_csrmm_f32(
    spmm_handle_t handle, int m, int n, int k, float alpha, const int* csrRowPtr,
    const int* csrColInd, const float* csrVal, int csrNnz, int blockDim, const int* bsrRowPtr,
    const int* bsrColInd, const float* bsrVal, int nnzb, const float* B, int ldb, float beta,
    float* C, int ldc) {
  // divide.cu:348-373 runs csrmm2 and bsrmm back to back with alpha = beta = 1
  // onto a zeroed C. Here the BSR part applies the caller's beta and the CSR
  // remainder accumulates on top, both on the handle's stream; with
  // fused (bs = 32) one launch does both per block row (§4a): by default when
  // the remainder averages <= 4096 entries per block row, or forced by flags.
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (m < 0 || n < 0 || k < 0 || csrNnz < 0 || nnzb < 0 || blockDim <= 0)
    return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!csrRowPtr || !C || ldb < n || ldc < n || (k > 0 && !B)) return SPMM_STATUS_INVALID_VALUE;
  if (nnzb > 0 && (!bsrRowPtr || !bsrColInd || !bsrVal)) return SPMM_STATUS_INVALID_VALUE;
  if (csrNnz > 0 && (!csrColInd || !csrVal)) return SPMM_STATUS_INVALID_VALUE;
  const int flags = handle->hybrid_flags;
  const bool want_fused =
      (flags & SPMM_HYBRID_FUSED) ||
      (!(flags & SPMM_HYBRID_TWO_LAUNCH) &&
       (int64_t)csrNnz <= kHybridFusedRemainderPerBlockRow * (int64_t)((m + 31) / 32));
  if (blockDim == 32 && nnzb > 0 && csrNnz > 0 && want_fused &&
      hybrid32_fusable(n, ldb, ldc, bsrVal, B, C))
    return launch_hybrid32_fused(handle, m, n, alpha, csrRowPtr, csrColInd, csrVal, bsrRowPtr,
                                 bsrColInd, bsrVal, B, ldb, beta, C, ldc);
  float csr_beta = beta;
  if (nnzb > 0) {
    const int mb = (m + blockDim - 1) / blockDim, kb = (k + blockDim - 1) / blockDim;
    spmm_status_t st = launch_bsrmm_f32(handle, SPMM_DIRECTION_ROW, mb, kb, n, nnzb, blockDim,
                                        alpha, bsrRowPtr, bsrColInd, bsrVal, B, ldb,
                                        SPMM_ORDER_ROW, beta, C, ldc, SPMM_ORDER_ROW,
                                        /*dense_blocks=*/true);
    if (st != SPMM_STATUS_SUCCESS) return st;
    csr_beta = 1.f;
  }
  return csrmm_impl(handle, m, n, k, csrNnz, alpha, csrRowPtr, csrColInd, csrVal, 0, B, ldb,
                    SPMM_ORDER_ROW, csr_beta, C, ldc, SPMM_ORDER_ROW);
}

// divide.cu's own call shape (divide.cu:218-230, 348-373): csrmm2 and bsrmm
// back to back onto one column-major z (ldc = nb*bs) with alpha = beta = 1,
// B column-major (transB = N, ldb = n) or row-major (transB = T, ldb = dim).
// Row-major B and C keep spmm_hybrid_csrmm_f32 (fused when it pays). Any
// column-major operand runs as two stream-ordered launches: a column-major B
// is transposed once into a row-major (ceil(k/bs)*bs) x n copy in the handle's
// scratch, zero rows past k (so the BSR part never reads past the caller's B:
// the reference's ldb = n is short of nb*bs when bs does not divide n); the
// BSR part runs the dense-block MFMA kernel on it, writing C in the caller's
// order through its own epilogue (beta), then the CSR remainder accumulates
// (beta = 1; a column-major C through the workspace transpose).
extern "C" spmm_status_t spmm_hybrid_csrmm_ex_f32(
    spmm_handle_t handle, int m, int n, int k, float alpha, const int* csrRowPtr,
    const int* csrColInd, const float* csrVal, int csrNnz, int blockDim, const int* bsrRowPtr,
    const int* bsrColInd, const float* bsrVal, int nnzb, const float* B, int ldb,
    spmm_order_t orderB, float beta, float* C, int ldc, spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (orderB == SPMM_ORDER_ROW && orderC == SPMM_ORDER_ROW)
    return spmm_hybrid_csrmm_f32(handle, m, n, k, alpha, csrRowPtr, csrColInd, csrVal, csrNnz,
                                 blockDim, bsrRowPtr, bsrColInd, bsrVal, nnzb, B, ldb, beta, C,
                                 ldc);
  if (m < 0 || n < 0 || k < 0 || csrNnz < 0 || nnzb < 0 || blockDim <= 0)
    return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!csrRowPtr || !C || (k > 0 && !B)) return SPMM_STATUS_INVALID_VALUE;
  if (nnzb > 0 && (!bsrRowPtr || !bsrColInd || !bsrVal)) return SPMM_STATUS_INVALID_VALUE;
  if (csrNnz > 0 && (!csrColInd || !csrVal)) return SPMM_STATUS_INVALID_VALUE;
  const int mb = (m + blockDim - 1) / blockDim, kb = (k + blockDim - 1) / blockDim;
  const long long rows_c = nnzb > 0 ? (long long)mb * blockDim : m;
  if (orderB == SPMM_ORDER_COL ? ldb < (k > 0 ? k : 1) : ldb < n) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_COL ? ldc < rows_c : ldc < n) return SPMM_STATUS_INVALID_VALUE;
  const float* Bx = B;
  int ldbx = ldb;
  if (orderB == SPMM_ORDER_COL && k > 0) {
    const size_t rows_b = nnzb > 0 ? (size_t)kb * blockDim : (size_t)k;
    spmm_status_t st = ensure_scratch(handle, rows_b * n * sizeof(float));
    if (st != SPMM_STATUS_SUCCESS) return st;
    float* Bt = static_cast<float*>(handle->scratch);
    // B (k x n col-major) is an (n x k) row-major matrix with ld ldb
    st = launch_transpose(handle, n, k, B, ldb, Bt, n, 0.f);
    if (st != SPMM_STATUS_SUCCESS) return st;
    if (rows_b > (size_t)k) {
      const hipError_t e = hipMemsetAsync(Bt + (size_t)k * n, 0,
                                          (rows_b - k) * n * sizeof(float), handle->stream);
      if (e != hipSuccess) return from_hip(e);
    }
    Bx = Bt;
    ldbx = n;
  }
  float csr_beta = beta;
  if (nnzb > 0) {
    spmm_status_t st = launch_bsrmm_f32(handle, SPMM_DIRECTION_ROW, mb, kb, n, nnzb, blockDim,
                                        alpha, bsrRowPtr, bsrColInd, bsrVal, Bx, ldbx,
                                        SPMM_ORDER_ROW, beta, C, ldc, orderC,
                                        /*dense_blocks=*/true);
    if (st != SPMM_STATUS_SUCCESS) return st;
    csr_beta = 1.f;
  }
  return csrmm_impl(handle, m, n, k, csrNnz, alpha, csrRowPtr, csrColInd, csrVal, 0, Bx, ldbx,
                    SPMM_ORDER_ROW, csr_beta, C, ldc, orderC);
}
