/*
 * spmm_hip.h — C ABI of the MI355X-native SpMM engine (libspmm_hip.so).
 *
 * This is the drop-in boundary for the two hot paths of
 * xuyifangreeneyes/spmm-denseblock:
 *
 *   Path A  CSR x dense   replaces gespmm_csrmm<T>          (gespmm_csrmm.h:422-426)
 *                          and the legacy cusparseScsrmm / cusparseScsrmm2 call
 *                          sites (run_csrmm.cu:133-142, test_csrmm.cu:126-129)
 *   Path B  BSR x dense   replaces rocsparse_bsrmm_template<T> (rocsparse_bsrmm.h:102-256)
 *                          and cusparseSbsrmm (run_bsrmm.cu:160-165), plus the
 *                          per-block cublasSgemm variant (block_cublas.cu:123-136)
 *   Prep    csr2bsr / bsr2csr / nnzb on the HOST (north_star: conversion stays
 *           CPU-side preprocessing), replacing cusparseXcsr2bsrNnz +
 *           cusparseScsr2bsr (run_bsrmm.cu:116-142) and cusparseSbsr2csr
 *           (bsr2csr.cu:186-188).
 *
 * Conventions
 *   - Plain C: pointers, sizes, enums. No HIP or torch types in signatures;
 *     a stream is passed as an opaque `void*` (a hipStream_t, 0 = default).
 *   - The caller owns every device buffer (the reference cudaMallocs in its
 *     drivers). Kernels never allocate; a handle may keep a small internal
 *     workspace (merge-path carries, layout staging) that it grows lazily.
 *   - Numeric values of spmm_status_t / spmm_direction_t / spmm_operation_t
 *     mirror cusparseStatus_t / cusparseDirection_t / cusparseOperation_t so a
 *     caller's HANDLE_CUSPARSE_ERROR-style checks keep working.
 *   - All index arrays are int32, as in the reference. fp32 values unless the
 *     function name says otherwise.
 */
#ifndef SPMM_HIP_H
#define SPMM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPMM_HIP_VERSION 100 /* 1.0.0 */

typedef enum {
  SPMM_STATUS_SUCCESS = 0,
  SPMM_STATUS_NOT_INITIALIZED = 1,
  SPMM_STATUS_ALLOC_FAILED = 2,
  SPMM_STATUS_INVALID_VALUE = 3,
  SPMM_STATUS_ARCH_MISMATCH = 4,
  SPMM_STATUS_MAPPING_ERROR = 5,
  SPMM_STATUS_EXECUTION_FAILED = 6,
  SPMM_STATUS_INTERNAL_ERROR = 7,
  SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED = 8,
  SPMM_STATUS_ZERO_PIVOT = 9,
  SPMM_STATUS_NOT_SUPPORTED = 10
} spmm_status_t;

typedef enum { SPMM_DIRECTION_ROW = 0, SPMM_DIRECTION_COLUMN = 1 } spmm_direction_t;

typedef enum {
  SPMM_OPERATION_NON_TRANSPOSE = 0,
  SPMM_OPERATION_TRANSPOSE = 1,
  SPMM_OPERATION_CONJUGATE_TRANSPOSE = 2
} spmm_operation_t;

/* Storage order of a dense matrix (explicit in the *_ex entry points). */
typedef enum { SPMM_ORDER_ROW = 0, SPMM_ORDER_COL = 1 } spmm_order_t;

typedef enum { SPMM_INDEX_BASE_ZERO = 0, SPMM_INDEX_BASE_ONE = 1 } spmm_index_base_t;

typedef enum { SPMM_MATRIX_TYPE_GENERAL = 0 } spmm_matrix_type_t;

typedef struct spmm_context* spmm_handle_t;    /* ~ cusparseHandle_t  */
typedef struct spmm_mat_descr* spmm_mat_descr_t; /* ~ cusparseMatDescr_t */

/* ------------------------------------------------------------------------ */
/* Handle / descriptor lifecycle (cusparseCreate, cusparseSetStream, ...)     */
/* ------------------------------------------------------------------------ */
int spmm_get_version(void);
const char* spmm_get_status_string(spmm_status_t status);

spmm_status_t spmm_create(spmm_handle_t* handle);
spmm_status_t spmm_destroy(spmm_handle_t handle);
spmm_status_t spmm_set_stream(spmm_handle_t handle, void* stream);
spmm_status_t spmm_get_stream(spmm_handle_t handle, void** stream);

spmm_status_t spmm_create_mat_descr(spmm_mat_descr_t* descr);
spmm_status_t spmm_destroy_mat_descr(spmm_mat_descr_t descr);
spmm_status_t spmm_set_mat_type(spmm_mat_descr_t descr, spmm_matrix_type_t type);
spmm_status_t spmm_set_mat_index_base(spmm_mat_descr_t descr, spmm_index_base_t base);

/* Per-launch device timing of the dominant kernel (hipEvents recorded on the
 * handle's stream around each main-kernel launch). Used by bench.py for the
 * roofline figure; off by default, costs two event records per launch. */
spmm_status_t spmm_set_kernel_timing(spmm_handle_t handle, int enable);
/* Synchronises the recorded events, returns up to max_count durations (ms),
 * oldest first, and clears the record. */
spmm_status_t spmm_get_kernel_times(spmm_handle_t handle, float* ms, int max_count, int* count);

/* Tuning knob for the CSR merge-path kernel: resident waves per CU the grid
 * is sized for (0 = default). */
spmm_status_t spmm_set_csr_waves_per_cu(spmm_handle_t handle, int waves_per_cu);
/* The target a handle without that setting sizes a CSR launch's grid for: 16
 * waves per CU, 12 from 2^20 rows on the plain kernel (hot != 0: the
 * spmm_csrmm_hot_f32 kernel, which keeps 16). Host-only; the result of the
 * product does not depend on it. */
int spmm_csr_default_waves_per_cu(int m, int hot);

/* CSR kernel options (bit flags). SPMM_CSR_NT_STREAMS: read colind/val and
 * write C with non-temporal hints, keeping L2 / MALL for the B gathers. */
#define SPMM_CSR_NT_STREAMS 1
/* K <= 32: use the one-nnz-per-wave-instruction kernel (one sequential FMA
 * chain per unsplit row, the reference's order) instead of the default
 * several-rows-per-instruction kernel (interleaved chains per row). */
#define SPMM_CSR_SEQUENTIAL_ROWS 2
spmm_status_t spmm_set_csr_options(spmm_handle_t handle, int flags);

/* BSR kernel options (bit flags, per handle).
 *
 * The default contract of the BSR entries at bs 16 / 32 (the column streams,
 * DESIGN.md §4) is COLUMN-GRANULAR: a column of a stored block whose values
 * are all +-0 is skipped; every other column multiplies whole, its explicit
 * zeros included. With finite B this is the dense block product exactly. With
 * an inf / NaN in B row J*bs + c, rows of block row I get a non-finite value
 * from it iff a stored block (I, J) holds a value other than +-0 in its
 * column c: then every row of block row I does (0 * inf = NaN for the rows
 * whose entry is an explicit zero), and if column c is all zeros none does.
 *
 * SPMM_BSR_DENSE_BLOCK_PRODUCT: cusparseSbsrmm's dense-block semantics
 * (bsrmm.cu:141-144): every stored block multiplies as a dense
 * bs x bs matrix, so an inf / NaN in B row J*bs + c reaches every row of every
 * block row that stores a block (I, J), whatever that block's column c holds.
 * Runs the full-panel kernels (bs 32 ROW blocks, row-major B: the LDS-staged
 * MFMA kernel the hybrid uses for dense blocks; otherwise the register-
 * fragment MFMA kernels) for spmm_bsrmm_ex_f32 / _f16, spmm_sbsrmm, the
 * analysed entries (which then ignore the masks) and the hybrid's BSR part.
 * Same result as the default on finite inputs, within the fp32 bar. */
#define SPMM_BSR_DENSE_BLOCK_PRODUCT 1
/* SPMM_BSR_SMALL_GROUPED: bs 2 / 4 / 8 (row-major B) take the grouped MFMA stream
 * (32 / bs block rows per wave share each B row of their column
 * union) whatever the matrix's size. By default it is taken from 2^20 stored
 * blocks up, where its fixed cost (a sharing probe and a block-row order,
 * about 40 us) is under a tenth of the product; below, and on matrices the probe
 * finds unshared, the lane-group VALU kernel runs. Same result bit for bit. */
#define SPMM_BSR_SMALL_GROUPED 2
spmm_status_t spmm_set_bsr_options(spmm_handle_t handle, int flags);

/* Which kernel the handle's last bs 2 / 4 / 8 fp32 product ran (a measurement
 * aid: the choice does not change the result): *path = 0 the lane-group VALU
 * kernel, 1 the grouped MFMA stream, 2 the grouped stream's branch whose
 * sharing probe gave the matrix to the lane-group kernel, -1 no such product
 * on this handle. Synchronises the handle's stream and reads the probe's sums
 * back; call it right after the product (the next product on the handle
 * reuses that scratch). */
spmm_status_t spmm_bsr_small_path(spmm_handle_t handle, int* path);

/* Build options of the loaded library (bit flags): SPMM_BUILD_TUNING is set
 * in an A/B build (make TUNING=1), whose kernel choice the environment may
 * override (SPMM_BSR_VARIANT, SPMM_BSR_ORDER, SPMM_CSR_GROUP_PD); a release
 * build reads no environment variable. */
#define SPMM_BUILD_TUNING 1
int spmm_get_build_options(void);

/* ------------------------------------------------------------------------ */
/* Path A: CSR x dense                                                         */
/* ------------------------------------------------------------------------ */

/* Drop-in for gespmm_csrmm<float> (gespmm_csrmm.h:422-426):
 *   C[A_nrows x B_ncols] = A(csr) * B, B and C row-major (ld = B_ncols),
 *   C overwritten (no alpha/beta), empty rows give 0. nnz is read from
 *   A_rowPtr[A_nrows] on the device. Runs on `stream` with a process-wide
 *   default handle. */
spmm_status_t spmm_gespmm_csrmm_f32(int A_nrows, int B_ncols, const int* A_rowPtr,
                                    const int* A_colInd, const float* A_val,
                                    const float* B, float* C, void* stream);

/* Drop-in for cusparseScsrmm (run_csrmm.cu:135-137):
 *   C(m x n, col-major, ldc) = alpha*op(A)(m x k) * B(k x n, col-major, ldb) + beta*C.
 * Only transA = NON_TRANSPOSE is supported (as in the reference call sites). */
spmm_status_t spmm_scsrmm(spmm_handle_t handle, spmm_operation_t transA, int m, int n, int k,
                          int nnz, const float* alpha, const spmm_mat_descr_t descrA,
                          const float* csrValA, const int* csrRowPtrA, const int* csrColIndA,
                          const float* B, int ldb, const float* beta, float* C, int ldc);

/* Drop-in for cusparseScsrmm2 (run_csrmm.cu:139-142, test_csrmm.cu:126-129):
 *   transB = NON_TRANSPOSE: B col-major k x n (ldb >= k);
 *   transB = TRANSPOSE:     B row-major k x n (ldb >= n);  C col-major. */
spmm_status_t spmm_scsrmm2(spmm_handle_t handle, spmm_operation_t transA,
                           spmm_operation_t transB, int m, int n, int k, int nnz,
                           const float* alpha, const spmm_mat_descr_t descrA,
                           const float* csrValA, const int* csrRowPtrA,
                           const int* csrColIndA, const float* B, int ldb,
                           const float* beta, float* C, int ldc);

/* General form with explicit dense storage orders (host-pointer alpha/beta).
 *   C(m x n) = alpha * A(m x k, csr) * B(k x n) + beta * C
 * orderB/orderC = SPMM_ORDER_ROW is the fast (native) layout; column-major
 * operands are staged through the handle workspace. beta == 0 never reads C. */
spmm_status_t spmm_csrmm_ex_f32(spmm_handle_t handle, int m, int n, int k, int nnz,
                                float alpha, const int* csrRowPtr, const int* csrColInd,
                                const float* csrVal, spmm_index_base_t base,
                                const float* B, int ldb, spmm_order_t orderB, float beta,
                                float* C, int ldc, spmm_order_t orderC);

/* Hot-column analysis for the CSR gathers (an extension, once per matrix like
 * cuSPARSE's SpMM preprocess; the reference's gespmm_csrmm.h / csrmm.cu have
 * none). Counts every column's nonzeros on the device and writes
 *   csrColIndHot[i] = csrColInd[i] | 0x80000000  if column csrColInd[i] is hot,
 *                     csrColInd[i]               otherwise,
 * hot = among the columns with the most nonzeros whose gathered B-row pieces
 * (n floats, at most one merge-path column tile) fit in hotBytes (0 = the
 * default below: half the 256-MB MALL). Requires column indices < 2^31 - 1.
 * The piece size assumes 16-B aligned B and C with ld % 4 == 0 (the layout
 * the kernel gathers 2 or 4 floats per lane from); with a misaligned B the
 * kernel gathers one float per lane and the hot set is up to 4x smaller than
 * hotBytes (results are unaffected: the tags are cache hints only).
 * Caller-owned output (nnz ints); scratch comes from the handle. The tagged
 * array is input for spmm_csrmm_hot_f32 only: every other entry reads it as
 * negative (out-of-range) column indices. */
#define SPMM_CSR_HOT_BYTES_DEFAULT (128ll << 20)
spmm_status_t spmm_csr_hot_analysis(spmm_handle_t handle, int n, int k, int nnz,
                                    const int* csrColInd, spmm_index_base_t base,
                                    long long hotBytes, int* csrColIndHot);

/* spmm_csrmm_ex_f32 on the tagged column indices of spmm_csr_hot_analysis:
 * hot columns' B rows are gathered with the default cache policy, every other
 * row non-temporal, so the long tail of rarely used rows does not evict the hub
 * rows from L2 and the MALL. Same arithmetic, order and result as
 * spmm_csrmm_ex_f32 on the untagged indices (bit-identical), same checks. */
spmm_status_t spmm_csrmm_hot_f32(spmm_handle_t handle, int m, int n, int k, int nnz,
                                 float alpha, const int* csrRowPtr, const int* csrColIndHot,
                                 const float* csrVal, spmm_index_base_t base, const float* B,
                                 int ldb, spmm_order_t orderB, float beta, float* C, int ldc,
                                 spmm_order_t orderC);

/* ------------------------------------------------------------------------ */
/* Path B: BSR x dense                                                         */
/* ------------------------------------------------------------------------ */

/* Drop-in for cusparseSbsrmm (run_bsrmm.cu:160-165) and, with alpha/beta
 * passed by pointer, rocsparse_bsrmm_template<float> (rocsparse_bsrmm.h:102-108):
 *   C(mb*bs x n, col-major, ldc) = alpha * A(bsr, mb x kb blocks) * op(B) + beta * C
 *   dir: block storage (ROW: val[b*bs*bs + r*bs + c]; COLUMN: val[b*bs*bs + c*bs + r])
 *   transB = NON_TRANSPOSE: B col-major (kb*bs x n, ldb >= kb*bs)
 *   transB = TRANSPOSE:     B row-major (kb*bs x n, ldb >= n)
 * Status behaviour follows rocsparse_bsrmm.h:109-176 (NOT_INITIALIZED for a
 * null handle, INVALID_VALUE for null descr / negative sizes / null pointers /
 * bad ld, MATRIX_TYPE_NOT_SUPPORTED for transA != N or a bad transB, SUCCESS
 * quick return when mb, n, kb or nnzb is 0). */
spmm_status_t spmm_sbsrmm(spmm_handle_t handle, spmm_direction_t dir,
                          spmm_operation_t transA, spmm_operation_t transB, int mb, int n,
                          int kb, int nnzb, const float* alpha, const spmm_mat_descr_t descrA,
                          const float* bsrValA, const int* bsrRowPtrA, const int* bsrColIndA,
                          int blockDim, const float* B, int ldb, const float* beta, float* C,
                          int ldc);

/* General form with explicit dense storage orders.
 *   C(mb*bs x n) = alpha * A(bsr) * B(kb*bs x n) + beta * C
 * bs in {16, 32} runs on fp32 MFMA (v_mfma_f32_{16x16x4,32x32x2}_f32); other
 * block sizes run a VALU kernel. The per-block cublasSgemm variant of
 * block_cublas.cu:123-136 is dir = COLUMN, orderB = ROW, orderC = COL, beta = 1. */
spmm_status_t spmm_bsrmm_ex_f32(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb,
                                int n, int nnzb, int blockDim, float alpha,
                                const int* bsrRowPtr, const int* bsrColInd,
                                const float* bsrVal, const float* B, int ldb,
                                spmm_order_t orderB, float beta, float* C, int ldc,
                                spmm_order_t orderC);

/* Analysis for the bs = 32 column stream (an extension: rocsparse_bsrmm.h:102-256
 * has no analysis step; this follows rocSPARSE's bsrmv analysis / cuSPARSE's
 * SpMM preprocess pattern). Once per matrix, on the handle's stream:
 *   masks[k]  bit c set iff column c of block k holds a value other than +-0
 *             (NaN and inf count), nnzb words;
 *   valCol    dir = ROW: a column-major copy of the blocks, nnzb * 1024 floats
 *             (may be null for dir = COLUMN, whose blocks already are).
 * Caller-owned buffers. INVALID_VALUE for a bad dir, nnzb < 0, a null
 * pointer that is needed, or a valCol that overlaps bsrVal (the analysis
 * reads whole blocks while it scatters their columns: no in-place form). */
spmm_status_t spmm_bsr32_analysis_f32(spmm_handle_t handle, spmm_direction_t dir, int nnzb,
                                      const float* bsrVal, unsigned* masks, float* valCol);

/* C(mb*32 x n) = alpha * A * B(kb*32 x n) + beta * C on the analysis: valCol are
 * the column-major blocks (valCol from spmm_bsr32_analysis_f32, or bsrVal of a
 * COLUMN-direction matrix) and masks their column masks. A column of a block
 * with no value other than +-0 is skipped, as the shipped column streams do; the
 * kernel reads only the nonzero columns' values. Same checks and quick returns
 * as spmm_bsrmm_ex_f32 with blockDim 32; layouts the analysed kernel cannot
 * take run the COLUMN-direction kernels on valCol. */
spmm_status_t spmm_bsrmm_analysed_f32(spmm_handle_t handle, int mb, int kb, int n, int nnzb,
                                      float alpha, const int* bsrRowPtr, const int* bsrColInd,
                                      const float* valCol, const unsigned* masks, const float* B,
                                      int ldb, spmm_order_t orderB, float beta, float* C,
                                      int ldc, spmm_order_t orderC);

/* The same analysis for bs = 16 fp16 blocks: masks[k] bit c (c < 16), and for
 * ROW blocks a column-major fp16 copy (nnzb * 256 halves); same checks. */
spmm_status_t spmm_bsr16_analysis_f16(spmm_handle_t handle, spmm_direction_t dir, int nnzb,
                                      const uint16_t* bsrVal, unsigned* masks, uint16_t* valCol);

/* C(mb*16 x n, fp32) = alpha * A * B(kb*16 x n, fp16) + beta * C on the bs = 16
 * analysis (fp16 A and B, fp32 accumulate), as spmm_bsrmm_ex_f16 with blockDim 16:
 * n >= 128 runs the analysed column stream, other shapes the COLUMN-direction
 * kernels on valCol. */
spmm_status_t spmm_bsrmm_analysed_f16(spmm_handle_t handle, int mb, int kb, int n, int nnzb,
                                      float alpha, const int* bsrRowPtr, const int* bsrColInd,
                                      const uint16_t* valCol, const unsigned* masks,
                                      const uint16_t* B, int ldb, spmm_order_t orderB,
                                      float beta, float* C, int ldc, spmm_order_t orderC);

/* The grouped bs = 16 fp16 stream (an extension, once per matrix like the
 * analyses above; DESIGN.md §4 "The grouped stream"). groupRows (2, 4 or 8;
 * 0 = the library's choice per matrix: the size query counts the items of
 * every W and keeps the one its time model ranks first, so a reordered graph
 * whose neighbouring rows share few columns gets 2; word 0 of the buffer holds
 * the W taken) adjacent block rows form a group whose waves share one copy of each
 * B row the union of their nonzero columns needs: on a reordered graph
 * neighbouring block rows need mostly the same rows (products stand-in: the
 * union is 0.43 of the (block row, column) pairs at 4 rows, 0.29 at 8).
 * Two phases: with buffer == NULL (the size query), *bufferBytes receives the
 * size of the caller-owned device buffer; with a buffer of that size the
 * analysis fills it. Everything runs on the device: the size query checks the
 * row pointer, counts and sums the groups' items there and synchronises the
 * handle's stream once (16 bytes come back for the size); the filling call
 * with the same arguments starts from the size query's device results, kept
 * on the handle, and only launches kernels and async copies (no
 * synchronisation, no host data: it can be captured in a HIP graph once the
 * handle's workspace has grown to the matrix). The arrays must not change
 * between the two calls (as between cuSPARSE's bufferSize and preprocess);
 * a filling call without a size query of the same arguments runs one first,
 * and every size query recomputes (a matrix at the addresses of an earlier
 * query is analysed afresh). Analyses on one handle from several threads run
 * one after the other (the handle's pending record is locked per call).
 * The handle records the buffer's layout:
 * spmm_bsrmm_grouped_f16 on the same handle takes it (until
 * spmm_bsr16_group_release or another analysis into the same buffer).
 * INVALID_VALUE for a bad dir / groupRows, negative sizes, null pointers that
 * are needed, a row pointer that does not run 0 .. nnzb, a negative block
 * column, block columns not strictly increasing within a block row (sorted,
 * no duplicates, as the csr2bsr output), or a short buffer; NOT_SUPPORTED
 * past 2^31 - 1 items. */
spmm_status_t spmm_bsr16_group_analysis_f16(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                            int nnzb, int groupRows, const int* bsrRowPtr,
                                            const int* bsrColInd, const uint16_t* bsrVal,
                                            void* buffer, size_t* bufferBytes);

/* C(mb*16 x n, fp32) = alpha * A * B(kb*16 x n, fp16) + beta * C on a group
 * analysis of A (fp32 accumulate), B row- or column-major (staged row-major),
 * C either order. Same sizes and ld checks as spmm_bsrmm_ex_f16;
 * INVALID_VALUE for a buffer this handle has no analysis of, another mb, or a
 * kb the analysed block columns do not fit (a column >= kb);
 * NOT_SUPPORTED when n % 8 != 0, a row-major ldb % 8 != 0 or B is not 16-B
 * aligned (spmm_bsrmm_ex_f16 serves those shapes). Non-finite B follows the
 * column-granular contract of the drop-in stream (spmm_set_bsr_options above):
 * each wave clears the B values of the entries its block row does not hold;
 * with finite B the product equals spmm_bsrmm_ex_f16's within the fp32 bar. */
spmm_status_t spmm_bsrmm_grouped_f16(spmm_handle_t handle, int mb, int kb, int n,
                                     const void* buffer, float alpha, const uint16_t* B, int ldb,
                                     spmm_order_t orderB, float beta, float* C, int ldc,
                                     spmm_order_t orderC);
/* The grouped bs = 32 fp32 stream (an extension, like the bs 16 one above;
 * DESIGN.md §4 "The grouped bs 32 stream"). groupRows 2 or 4 (0 = 2) adjacent
 * block rows share one copy of each B row of their union; unlike bs 16 each
 * block row multiplies only its own nonzero columns (the analysis records them
 * per item), so C is bit-identical to spmm_bsrmm_ex_f32 /
 * spmm_bsrmm_analysed_f32 with the same column-granular non-finite contract.
 * Same two phases, checks and handle record as spmm_bsr16_group_analysis_f16.
 * The analysis reads A once: for ROW blocks the size query keeps a compact copy
 * of the blocks' nonzero columns in a stream-ordered allocation of 4 KB per block
 * (at most 16 GiB and a quarter of the free device memory)
 * (hipMallocAsync on the handle's stream), which the filling call reads and frees;
 * a filling call under stream capture reads the values instead and leaves the
 * copy to the next size query or spmm_destroy. Without memory for the copy the
 * filling call reads the blocks themselves; the buffer's bytes are the same. */
spmm_status_t spmm_bsr32_group_analysis_f32(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                            int nnzb, int groupRows, const int* bsrRowPtr,
                                            const int* bsrColInd, const float* bsrVal,
                                            void* buffer, size_t* bufferBytes);

/* C(mb*32 x n) = alpha * A * B(kb*32 x n) + beta * C on a bs 32 group analysis of A,
 * B and C row- or column-major (column-major ones are staged row-major in the
 * workspace). INVALID_VALUE as spmm_bsrmm_grouped_f16 (a bs 16 analysis is not
 * taken); NOT_SUPPORTED when n % 4 != 0, a row-major ldb or ldc % 4 != 0, or B or
 * C is not 16-B aligned (spmm_bsrmm_ex_f32 serves those shapes). */
spmm_status_t spmm_bsrmm_grouped_f32(spmm_handle_t handle, int mb, int kb, int n,
                                     const void* buffer, float alpha, const float* B, int ldb,
                                     spmm_order_t orderB, float beta, float* C, int ldc,
                                     spmm_order_t orderC);

/* Forgets the handle's record of a group-analysis buffer, bs 16 or bs 32 (before
 * freeing it). spmm_bsr_group_release is the same call under a block-size-neutral
 * name; spmm_bsr16_group_release stays for the bs 16 stream's first users. */
spmm_status_t spmm_bsr_group_release(spmm_handle_t handle, const void* buffer);
spmm_status_t spmm_bsr16_group_release(spmm_handle_t handle, const void* buffer);

/* fp16 A and B (IEEE binary16 bit patterns), fp32 accumulate and fp32 C.
 * bs = 16 runs on v_mfma_f32_16x16x32_f16 with two blocks per instruction. */
spmm_status_t spmm_bsrmm_ex_f16(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb,
                                int n, int nnzb, int blockDim, float alpha,
                                const int* bsrRowPtr, const int* bsrColInd,
                                const uint16_t* bsrVal, const uint16_t* B, int ldb,
                                spmm_order_t orderB, float beta, float* C, int ldc,
                                spmm_order_t orderC);

/* Re-blocking to bs 32 on the device (an extension; DESIGN.md §4, "Small blocks
 * re-blocked to 32"): the same matrix in 32 x 32 blocks, so a bs = 2 / 4 / 8 / 16
 * product can run on the bs 32 MFMA streams (spmm_bsr32_analysis_f32 +
 * spmm_bsrmm_analysed_f32, or the group analysis) instead of the VALU kernel.
 * A block (I, J) of blockDim lands in block (I / R, J / R), R = 32 / blockDim, at
 * sub-block (I % R, J % R); the rest of each 32 x 32 block is zero. dir is kept
 * (ROW blocks stay ROW). mb32 = ceil(mb / R) block rows; the product then needs
 * B with ceil(kb / R) * 32 rows and C with mb32 * 32 rows (the extra rows are
 * zero columns / rows of A). cusparseXcsr2bsrNnz / Scsr2bsr's two calls: the
 * first fills bsrRowPtr32[mb32 + 1] and *nnzb32HostPtr (it synchronises the
 * handle's stream), the second bsrColInd32[nnzb32] and bsrVal32[nnzb32 * 1024]
 * (zero-filled first; no synchronisation). Block columns must be sorted per
 * block row; a negative one is INVALID_VALUE. */
spmm_status_t spmm_xbsr_reblock32_nnzb(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                       int nnzb, int blockDim, const int* bsrRowPtr,
                                       const int* bsrColInd, int* bsrRowPtr32,
                                       int* nnzb32HostPtr);
spmm_status_t spmm_sbsr_reblock32(spmm_handle_t handle, spmm_direction_t dir, int mb, int nnzb,
                                  int blockDim, const int* bsrRowPtr, const int* bsrColInd,
                                  const float* bsrVal, const int* bsrRowPtr32, int nnzb32,
                                  int* bsrColInd32, float* bsrVal32);

/* ------------------------------------------------------------------------ */
/* Preprocessing on the HOST (all pointers are host pointers)                  */
/* ------------------------------------------------------------------------ */

/* cusparseXcsr2bsrNnz semantics (run_bsrmm.cu:121-131): fills
 * bsrRowPtr[mb+1] (mb = ceil(m/blockDim)) and *nnzbTotal. */
spmm_status_t spmm_xcsr2bsr_nnz(spmm_direction_t dir, int m, int n, const int* csrRowPtr,
                                const int* csrColInd, int blockDim, int* bsrRowPtr,
                                int* nnzbTotal);

/* cusparseScsr2bsr semantics (run_bsrmm.cu:136-142): bsrRowPtr must come from
 * spmm_xcsr2bsr_nnz; bsrColInd[nnzb] sorted per block row; bsrVal[nnzb*bs*bs]
 * zero-filled, values placed per `dir`. Duplicate (row, col) entries are
 * summed. */
spmm_status_t spmm_scsr2bsr(spmm_direction_t dir, int m, int n, const float* csrVal,
                            const int* csrRowPtr, const int* csrColInd, int blockDim,
                            const int* bsrRowPtr, float* bsrVal, int* bsrColInd);

/* cusparseSbsr2csr semantics (bsr2csr.cu:177-188): every block expanded,
 * explicit zeros kept: nnz = nnzb*bs*bs, csrRowPtr[mb*bs+1]. */
spmm_status_t spmm_sbsr2csr(spmm_direction_t dir, int mb, int nb, const float* bsrVal,
                            const int* bsrRowPtr, const int* bsrColInd, int blockDim,
                            float* csrVal, int* csrRowPtr, int* csrColInd);

/* calculateNnzb (utility.cc:47-69) over a CSR pattern: number of nonzero
 * bs x bs blocks. */
int64_t spmm_calculate_nnzb(int n, const int* csrRowPtr, const int* csrColInd, int blockDim);

/* nnz-balanced contiguous row partition for multi-GPU sharding:
 * bounds[0] = 0, bounds[nparts] = m, part p owns rows [bounds[p], bounds[p+1]).
 * Minimises the max over parts of (nnz + rows) by a prefix search on rowptr. */
spmm_status_t spmm_csr_partition_rows(int m, const int* csrRowPtr, int nparts, int* bounds);

/* divide_matrix (divide.cu:52-127), with values: the n x n CSR is split into
 * a BSR part (DIRECTION_ROW) holding every bs x bs block whose fill
 * (entries / bs^2) is >= density, and a CSR remainder holding the other
 * entries in their original order. As in the reference, density <= 0 admits
 * every block, empty ones included (divide.cu:91). Host pointers, two
 * phases: sizes (csrRowPtr[n+1], bsrRowPtr[mb+1], totals), then fill.
 * Duplicate entries inside a BSR block are summed. */
spmm_status_t spmm_divide_nnz(int n, const int* rowPtr, const int* colInd, int blockDim,
                              float density, int* csrRowPtr, int* bsrRowPtr, int* csrNnz,
                              int* nnzb);
spmm_status_t spmm_sdivide(int n, const int* rowPtr, const int* colInd, const float* val,
                           int blockDim, float density, const int* csrRowPtr,
                           const int* bsrRowPtr, int* csrColInd, float* csrVal, int* bsrColInd,
                           float* bsrVal);

/* Device-pointer conversions: the argument order and
 * meaning of cusparseXcsr2bsrNnz / cusparseScsr2bsr (run_bsrmm.cu:121-142) and
 * cusparseSbsr2csr (bsr2csr.cu:186-188), on the handle's stream. The index
 * bases come from the descriptors. csr2bsr needs rows sorted by column (the
 * csrSorted* contract) and blockDim <= 64; duplicates are summed in CSR
 * order, so every output is bit-identical to the host conversions above.
 * nnzTotalHostPtr is a host pointer (the call synchronises, as cuSPARSE's host
 * pointer mode does); a column outside [0, n) makes it return
 * SPMM_STATUS_INVALID_VALUE. csr2bsr zero-fills bsrVal itself. */
spmm_status_t spmm_xcsr2bsr_nnz_dev(spmm_handle_t handle, spmm_direction_t dir, int m, int n,
                                    const spmm_mat_descr_t descrA, const int* csrRowPtr,
                                    const int* csrColInd, int blockDim,
                                    const spmm_mat_descr_t descrC, int* bsrRowPtr,
                                    int* nnzTotalHostPtr);
spmm_status_t spmm_scsr2bsr_dev(spmm_handle_t handle, spmm_direction_t dir, int m, int n,
                                const spmm_mat_descr_t descrA, const float* csrVal,
                                const int* csrRowPtr, const int* csrColInd, int blockDim,
                                const spmm_mat_descr_t descrC, float* bsrVal,
                                const int* bsrRowPtr, int* bsrColInd);
spmm_status_t spmm_sbsr2csr_dev(spmm_handle_t handle, spmm_direction_t dir, int mb, int nb,
                                const spmm_mat_descr_t descrA, const float* bsrVal,
                                const int* bsrRowPtr, const int* bsrColInd, int blockDim,
                                const spmm_mat_descr_t descrC, float* csrVal, int* csrRowPtr,
                                int* csrColInd);

/* cusparseXcoo2csr (csrmm.cu:148-149): csrRowPtr[m+1] of a COO whose row
 * indices cooRowInd[nnz] are sorted ascending (device pointers, handle's
 * stream). Row indices and the output are in idxBase, as in cuSPARSE:
 * csrRowPtr[0] = idxBase, csrRowPtr[m] = nnz + idxBase. */
spmm_status_t spmm_xcoo2csr(spmm_handle_t handle, const int* cooRowInd, int nnz, int m,
                            int* csrRowPtr, spmm_index_base_t idxBase);

/* Threshold planner for divide (the reference takes `density` from the user,
 * divide.cu:348): from the histogram of block fills it picks the count
 * threshold T minimising a bytes-over-bandwidth model of the hybrid SpMM,
 *   sum_{blocks, fill >= T} (s*(bs^2 + bs*K) + 4) / bsrBytesPerSec
 * + sum_{blocks, fill <  T} fill * (8 + 4*K)    / csrBytesPerSec,
 * s = valueBytes of the BSR part, and returns density = T / bs^2 (the value
 * spmm_divide_nnz admits exactly those blocks for; T = bs^2 + 1 means "all
 * CSR"). Bandwidths <= 0 take the defaults measured on MI355X with this
 * library (BSR 7.0e12, CSR 7.5e12 algorithmic bytes/s).
 * nnzb / csrNnz / estSeconds: the split and modelled time (may be NULL). */
spmm_status_t spmm_hybrid_plan(int n, const int* rowPtr, const int* colInd, int blockDim, int K,
                               int valueBytes, double bsrBytesPerSec, double csrBytesPerSec,
                               float* density, int64_t* nnzb, int64_t* csrNnz,
                               double* estSeconds);

/* ------------------------------------------------------------------------ */
/* fp64 (T = double in gespmm_csrmm<T> / rocsparse_bsrmm_template<T>,          */
/* gespmm_csrmm.h:422, rocsparse_bsrmm.h:102): same semantics and checks as    */
/* the fp32 entry points, VALU fp64 kernels (one sequential FMA chain per CSR  */
/* output element in CSR order).                                              */
/* ------------------------------------------------------------------------ */
spmm_status_t spmm_gespmm_csrmm_f64(int A_nrows, int B_ncols, const int* A_rowPtr,
                                    const int* A_colInd, const double* A_val, const double* B,
                                    double* C, void* stream);
spmm_status_t spmm_csrmm_ex_f64(spmm_handle_t handle, int m, int n, int k, int nnz, double alpha,
                                const int* csrRowPtr, const int* csrColInd, const double* csrVal,
                                spmm_index_base_t base, const double* B, int ldb,
                                spmm_order_t orderB, double beta, double* C, int ldc,
                                spmm_order_t orderC);
/* cusparseDcsrmm2 */
spmm_status_t spmm_dcsrmm2(spmm_handle_t handle, spmm_operation_t transA,
                           spmm_operation_t transB, int m, int n, int k, int nnz,
                           const double* alpha, const spmm_mat_descr_t descrA,
                           const double* csrValA, const int* csrRowPtrA, const int* csrColIndA,
                           const double* B, int ldb, const double* beta, double* C, int ldc);
spmm_status_t spmm_bsrmm_ex_f64(spmm_handle_t handle, spmm_direction_t dir, int mb, int kb, int n,
                                int nnzb, int blockDim, double alpha, const int* bsrRowPtr,
                                const int* bsrColInd, const double* bsrVal, const double* B,
                                int ldb, spmm_order_t orderB, double beta, double* C, int ldc,
                                spmm_order_t orderC);
/* cusparseDbsrmm / rocsparse_bsrmm_template<double> */
spmm_status_t spmm_dbsrmm(spmm_handle_t handle, spmm_direction_t dir, spmm_operation_t transA,
                          spmm_operation_t transB, int mb, int n, int kb, int nnzb,
                          const double* alpha, const spmm_mat_descr_t descrA,
                          const double* bsrValA, const int* bsrRowPtrA, const int* bsrColIndA,
                          int blockDim, const double* B, int ldb, const double* beta, double* C,
                          int ldc);

/* ------------------------------------------------------------------------ */
/* Hybrid dense-block + CSR-remainder SpMM (divide.cu:348-373)                */
/* ------------------------------------------------------------------------ */

/* Hybrid options (per handle). At bs = 32 the hybrid runs either fused, in
 * one launch (MFMA part, then each block row's CSR remainder in the same
 * workgroup), or as two stream-ordered launches (BSR kernel, then the CSR
 * kernel with beta = 1). Same result up to the CSR kernel's split-row carries.
 * By default (flags 0) it is fused when the remainder averages at most 4096
 * entries per block row (csrNnz <= 4096 * mb); longer per-block-row
 * remainders keep the merge-path CSR kernel's balance. SPMM_HYBRID_FUSED / SPMM_HYBRID_TWO_LAUNCH force
 * one form. */
#define SPMM_HYBRID_FUSED 1
#define SPMM_HYBRID_TWO_LAUNCH 2
/* Opt-in: the bs = 32 dense-block part computes each fp32 product as six
 * bf16 MFMA products of an exact three-way bf16 split of A and B (dropped
 * terms < 2^-21 |a||b| per product; accumulation in fp32). DESIGN.md §4a.
 * Inf and NaN inputs pass through the high part (the lower parts are zeroed),
 * so non-finite values propagate as in the fp32 path. The flag takes effect
 * only on the bs = 32 LDS-staged forms: the fused launch, and the two-launch
 * BSR part when n % 4 == 0, ldb % 4 == 0 and B / bsrVal are 16-byte aligned;
 * elsewhere (bs != 32, other layouts) the
 * dense-block part runs the plain fp32 MFMA kernel, with the same result
 * within the fp32 bar. */
#define SPMM_HYBRID_SPLIT_BF16 4
spmm_status_t spmm_set_hybrid_options(spmm_handle_t handle, int flags);

/* C(m x n) = alpha * (A_bsr + A_csr) * B(k x n) + beta * C, row-major B and C.
 * A_bsr is the BSR part of spmm_sdivide (bs x bs blocks, mb = ceil(m/bs)
 * block rows), A_csr the remainder. When nnzb > 0, B must hold
 * ceil(k/bs)*bs rows and C ceil(m/bs)*bs rows (padded, as the reference's
 * drivers allocate them, run_bsrmm.cu:86-94). The BSR part runs on MFMA
 * (writing C with beta), then the CSR part accumulates (beta = 1). */
spmm_status_t spmm_hybrid_csrmm_f32(spmm_handle_t handle, int m, int n, int k, float alpha,
                                    const int* csrRowPtr, const int* csrColInd,
                                    const float* csrVal, int csrNnz, int blockDim,
                                    const int* bsrRowPtr, const int* bsrColInd,
                                    const float* bsrVal, int nnzb, const float* B, int ldb,
                                    float beta, float* C, int ldc);

/* The same with explicit storage orders: divide.cu's own call shape
 * (divide.cu:218-230, 348-373) is csrmm2 + bsrmm onto a column-major z
 * (ldc = nb*bs) with alpha = beta = 1, B column-major (transB = N, ldb >= k)
 * or row-major (transB = T, ldb >= n). Row-major B and C are
 * spmm_hybrid_csrmm_f32. Otherwise two stream-ordered launches: a
 * column-major B is transposed once into the handle's scratch (zero rows
 * past k, so ldb need only cover the k real rows), the BSR part writes C in
 * orderC with beta, then the CSR remainder accumulates. A column-major C
 * needs ldc >= ceil(m/bs)*bs when nnzb > 0 (>= m otherwise). */
spmm_status_t spmm_hybrid_csrmm_ex_f32(spmm_handle_t handle, int m, int n, int k, float alpha,
                                       const int* csrRowPtr, const int* csrColInd,
                                       const float* csrVal, int csrNnz, int blockDim,
                                       const int* bsrRowPtr, const int* bsrColInd,
                                       const float* bsrVal, int nnzb, const float* B, int ldb,
                                       spmm_order_t orderB, float beta, float* C, int ldc,
                                       spmm_order_t orderC);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SPMM_HIP_H */
