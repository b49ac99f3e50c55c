// context.hpp — internal state behind spmm_handle_t / spmm_mat_descr_t.
//
// The reference has no handle of its own: gespmm_csrmm<T> launches on the
// legacy default stream (gespmm_csrmm.h:401-405) and the cuSPARSE paths use a
// cusparseHandle_t created in each driver (run_csrmm.cu:104). Here the handle
// carries the stream, a lazily grown device workspace (merge-path carries and
// column-major staging), the device's CU count for grid sizing, and an
// optional ring of hipEvent pairs used to time the dominant kernel.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <vector>

#include "spmm_hip.h"

struct spmm_mat_descr {
  spmm_matrix_type_t type = SPMM_MATRIX_TYPE_GENERAL;
  spmm_index_base_t base = SPMM_INDEX_BASE_ZERO;
};

struct spmm_context {
  hipStream_t stream = nullptr;
  int device = 0;
  int num_cus = 256;
  int csr_waves_per_cu = 0;  // 0 = default
  int csr_flags = SPMM_CSR_NT_STREAMS;  // SPMM_CSR_* option bits (default: nt streams)
  int hybrid_flags = 0;                 // SPMM_HYBRID_* option bits
  int bsr_flags = 0;                    // SPMM_BSR_* option bits
  // the last bs 2 / 4 / 8 fp32 product: -1 none, 0 the lane-group kernel, 1 the
  // grouped stream's branch (its probe's sums, left at scratch[0..15], decide)
  int small_path = -1, small_path_bs = 0;

  // Device workspace (grown, never shrunk; freed in spmm_destroy).
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // Kernel scratch (item records, segment partial tiles), apart from ws: ws may
  // hold a staged (transposed) B that the kernel reading it must not overwrite.
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // Block-row order of the column-stream BSR kernels (mb ints, grown like ws).
  int* order = nullptr;
  size_t order_cap = 0;
  // Split-row tickets of the CSR kernels (one int per merge-path slot): zero
  // between launches (each launch's last arrival resets what it counted), so
  // they live apart from ws, which other entries overwrite.
  int* tickets = nullptr;
  size_t tickets_cap = 0;
  // Group analyses made on this handle (spmm_bsr16_group_analysis_f16 /
  // spmm_bsr32_group_analysis_f32): buffer -> its shape, so the grouped product needs
  // no device read to size its grid.
  struct GroupPlan {
    int W, mb, ngroups;
    long long nitems;
    size_t bytes, rows_off, afrag_off;
    int max_col;  // largest block column (-1: none), checked against kb
    int bs = 16;  // 16: fp16 analysis; 32: fp32 analysis (wmask_off used)
    size_t wmask_off = 0;
  };
  std::map<const void*, GroupPlan> group_plans;
  // The size query of a group analysis (buffer == NULL) leaves its device results
  // (column masks, item pointers) in grp_pend for the filling call with the same
  // arguments, which then needs neither those kernels again nor any host round trip
  // (group.cpp). Every size query recomputes it (the arrays' contents may have
  // changed at the same addresses); the filling call consumes it. grp_mu holds
  // the record for a whole analysis call, so two threads analysing on one handle
  // run one after the other.
  struct GroupPending {
    bool valid = false;
    int bs = 0, W = 0, req = -1, dir = 0, mb = 0, nnzb = 0;  // req: the caller's groupRows
    const void *rp = nullptr, *ci = nullptr, *val = nullptr;
    long long nitems = 0;
    int max_col = -1;
    size_t need = 0, rows_off = 0, wmask_off = 0, afrag_off = 0;
    size_t ptr_off = 0;  // offset of the item pointers in grp_pend (masks at 0)
  };
  GroupPending grp_pending;
  void* grp_pend = nullptr;
  size_t grp_pend_bytes = 0;
  // the compact column copy of a pending bs 32 ROW analysis (4 KB per block, stream-ordered
  // allocation): freed by the filling call that uses it, or by the next size query
  void* grp_cols = nullptr;
  std::mutex grp_mu;

  // Kernel timing ring.
  bool timing = false;
  std::vector<hipEvent_t> ev_start, ev_stop;
  size_t ev_used = 0;

  std::mutex mu;  // serialises workspace growth for the shared default handle
};

namespace spmm {

// Grow the handle workspace to at least `bytes`. Not graph-capture safe on
// the first (growing) call; steady-state calls never allocate.
spmm_status_t ensure_workspace(spmm_context* ctx, size_t bytes);
// The same for the kernel scratch buffer.
spmm_status_t ensure_scratch(spmm_context* ctx, size_t bytes);
// The same for the block-row order buffer (at least n ints).
spmm_status_t ensure_order_buffer(spmm_context* ctx, size_t n);
// The same for the pending group analysis (grp_pend).
spmm_status_t ensure_group_pending(spmm_context* ctx, size_t bytes);
// At least n zeroed ticket words (zeroed on the handle's stream when grown).
spmm_status_t ensure_tickets(spmm_context* ctx, size_t n);

// Record a start/stop event pair around the next main-kernel launch when
// timing is on. Returns the pair index or -1.
int timing_begin(spmm_context* ctx);
void timing_end(spmm_context* ctx, int slot);

// Process-wide default handle for the handle-less gespmm entry point.
spmm_context* default_context();

inline spmm_status_t from_hip(hipError_t e) {
  if (e == hipSuccess) return SPMM_STATUS_SUCCESS;
  if (e == hipErrorOutOfMemory) return SPMM_STATUS_ALLOC_FAILED;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return SPMM_STATUS_ARCH_MISMATCH;
  return SPMM_STATUS_EXECUTION_FAILED;
}

// Kernel launchers (csr_kernels.hip / bsr_kernels.hip). Pointers are device
// pointers; all shape checks have been done by the API layer.
// carry_ws: csrmm_carry_bytes of workspace (split-row partials, rewritten by
// every launch); the split-row tickets come from ensure_tickets.
spmm_status_t launch_csrmm_rowmajor(spmm_context* ctx, int m, int n, const int* rowptr,
                                    const int* colind, const float* val, int base,
                                    const float* B, int ldb, float alpha, float beta, float* C,
                                    int ldc, void* carry_ws, int nnz_hint,
                                    int hot = 0);  // 1: hot-tagged colind; 2: and B below 4 GB
// spmm_csr_hot_analysis: colind_out = colind with bit 31 set on hot columns
spmm_status_t launch_csr_hot_analysis(spmm_context* ctx, int k, long long nnz, const int* colind,
                                      int base, long long hot_rows, int* colind_out);
size_t csrmm_carry_bytes(spmm_context* ctx, int m, int n);

spmm_status_t launch_transpose16(spmm_context* ctx, int rows, int cols, const uint16_t* src,
                                 int ld_src, uint16_t* dst, int ld_dst);
spmm_status_t launch_transpose(spmm_context* ctx, int rows, int cols, const float* src,
                               int ld_src, float* dst, int ld_dst, float beta);

spmm_status_t launch_bsrmm_f32(spmm_context* ctx, spmm_direction_t dir, int mb, int kb, int n,
                               int nnzb, int bs, float alpha, const int* rowptr,
                               const int* colind, const float* val, const float* B, int ldb,
                               spmm_order_t orderB, float beta, float* C, int ldc,
                               spmm_order_t orderC, bool dense_blocks = false,
                               const unsigned* masks = nullptr);
// spmm_bsr32_analysis_f32: column masks (+ a column-major copy of ROW blocks)
spmm_status_t launch_bsr32_analysis(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                    const float* val, unsigned* masks, float* val_col);

// Fused hybrid (bs = 32, row-major B and C): one launch, BSR MFMA part plus the
// CSR remainder per block row (bsr_kernels.hip). C holds ceil(m/32)*32 rows.
bool hybrid32_fusable(int n, int ldb, int ldc, const float* bval, const float* B, const float* C);
spmm_status_t launch_hybrid32_fused(spmm_context* ctx, int m, int n, float alpha,
                                    const int* crp, const int* cci, const float* cv,
                                    const int* brp, const int* bci, const float* bval,
                                    const float* B, int ldb, float beta, float* C, int ldc);
spmm_status_t launch_csrmm_f64(spmm_context* ctx, int m, int n, const int* rowptr,
                               const int* colind, const double* val, int base, const double* B,
                               int ldb, bool brow, double alpha, double beta, double* C, int ldc,
                               bool crow);
spmm_status_t launch_bsrmm_f64(spmm_context* ctx, spmm_direction_t dir, int mb, int n, int bs,
                               const int* rowptr, const int* colind, const double* val,
                               const double* B, int ldb, bool brow, double alpha, double beta,
                               double* C, int ldc, bool crow);
spmm_status_t launch_bsrmm_f16(spmm_context* ctx, spmm_direction_t dir, int mb, int kb, int n,
                               int nnzb, int bs, float alpha, const int* rowptr,
                               const int* colind, const uint16_t* val, const uint16_t* B,
                               int ldb, spmm_order_t orderB, float beta, float* C, int ldc,
                               spmm_order_t orderC, const unsigned* masks = nullptr);
spmm_status_t launch_bsr16_analysis(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                    const uint16_t* val, unsigned* masks, uint16_t* val_col);
// the grouped bs 16 stream: A-fragment fill (analysis) and the product
spmm_status_t launch_bsr16_grp_fill(spmm_context* ctx, long long nitems, int W, spmm_direction_t dir,
                                    const int* rows, const int* src, const uint16_t* val,
                                    unsigned* afrag);
spmm_status_t launch_bsrmm_grouped_f16(spmm_context* ctx, int W, int mb, int n, int ngroups,
                                       const int* item_ptr, const int* rows,
                                       const unsigned* wmask, const unsigned* afrag,
                                       const uint16_t* B16, int ldb, float alpha, float beta,
                                       float* C, int ldc, bool crow);
// the group analyses' device merge (group_kernels.hip; grp_build_kernel: PASS 1 checks
// the row pointer and the block columns and counts, PASS 2 writes the entries), the
// per-(item, wave) masks of held entries from the written sources
spmm_status_t launch_grp_build(spmm_context* ctx, int W, int BS, bool pass2, int mb, int nnzb,
                               int ngroups, const int* rp, const int* ci, const unsigned* mk,
                               int* cnt, int* maxj, const int* item_ptr, int* rows, int* src);
spmm_status_t launch_grp_wmask(spmm_context* ctx, long long nitems, int W, int E, const int* src,
                               unsigned* wmask);
// the bs 16 column masks of the group analysis (16-B aligned values; masks only)
spmm_status_t launch_grp_mask16(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                const uint16_t* val, unsigned* masks);
// stats[0] = max over maxj[0..n), stats[1] = 1 if any maxj is INT_MIN (pass 1's "bad")
spmm_status_t launch_grp_stats(spmm_context* ctx, const int* maxj, int n, int* stats);
// exclusive scan of count[0..n) into out[0..n] (out[0] = 0) and *total (one workgroup,
// convert_kernels.hip)
spmm_status_t launch_scan_counts(spmm_context* ctx, const int* count, int n, int* out,
                                 long long* total);
// the grouped bs 32 stream (row-major B and C)
spmm_status_t launch_bsr32_grp_fill(spmm_context* ctx, long long nitems, int W, spmm_direction_t dir,
                                    const int* rows, const int* src, const float* val,
                                    float* afrag);
// the bs 32 group analysis in one pass over A: masks plus the compact column copy of ROW
// blocks (cols: nnzb * 1024 floats, or null), and the fill from those columns (masks: the
// compact copy's ranks; null: cols = the COLUMN blocks' own values)
spmm_status_t launch_grp_mask32(spmm_context* ctx, spmm_direction_t dir, int nnzb, const float* val,
                                unsigned* masks, float* cols);
spmm_status_t launch_bsr32_grp_fillc(spmm_context* ctx, long long nitems, int W, const int* rows,
                                     const int* src, const float* cols, const unsigned* masks,
                                     float* afrag);
spmm_status_t launch_bsrmm_grouped_f32(spmm_context* ctx, int W, int mb, int n, int ngroups,
                                       const int* item_ptr, const int* rows,
                                       const unsigned* wmask, const float* afrag, const float* B,
                                       int ldb, float alpha, float beta, float* C, int ldc);

}  // namespace spmm
