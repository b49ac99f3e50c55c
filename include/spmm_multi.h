/*
 * spmm_multi.h — single-process multi-GPU CSR x dense over RCCL
 * (libspmm_hip.so; SURVEY.md §8b "spmm_csr_f32_multi", §8e; BASELINE.json
 * configs[3]: row-partitioned ogbn-products K = 256 + RCCL all-gather).
 *
 * The reference has no multi-GPU code: this is the
 * capability BASELINE config 4 names, behind the same plain-C conventions as
 * spmm_hip.h. One host thread drives every GPU of the node: one RCCL
 * communicator per device (ncclCommInitAll), one compute stream and one
 * collective stream per device, one spmm handle per device.
 *
 * Partitioning (host, spmm_csr_partition_rows in spmm_hip.h): contiguous row
 * ranges of A balanced on nnz + rows, part p = rows [bounds[p], bounds[p+1]).
 * B is replicated (2.5 GB for products at K = 256 against 288 GB of HBM per
 * GPU). Each device computes its rows straight into the same rows of its own
 * C, and the rows are exchanged over xGMI with grouped ncclSend / ncclRecv
 * (an all-gather of exact, uneven shards: every peer pair on its own link),
 * so every device ends up holding all of C.
 *
 * Output layout on every device: the m x n row-major C itself, leading
 * dimension ldc. Part p's local rows are cut into chunks of chunkRows =
 * spmm_multi_slot_rows(...) rows; with chunks > 1 the exchange of chunk c
 * (collective stream) runs while chunk c+1 is computed. The exchange moves
 * each chunk as one contiguous span of rows, so with ngpu > 1 C must be
 * packed (ldc == n; SPMM_STATUS_NOT_SUPPORTED otherwise): padding columns
 * between rows would travel with them and overwrite the caller's.
 *
 * Numerics: each device runs the 1-GPU kernel on its rows, and the kernels
 * associate a row's sum by the row alone (pieces from the row's start,
 * DESIGN.md §3c), so C is bit-identical to spmm_csrmm_ex_f32 on the whole
 * matrix for any ngpu, bounds and chunks — at n <= 64 (the lane-group
 * kernel, whose chains follow array positions mod 64) when part p's arrays
 * keep the whole matrix's nonzero positions mod 64 (views into the whole
 * arrays, or copies offset as spmm_hip.dist.make_shard does).
 */
#ifndef SPMM_MULTI_H
#define SPMM_MULTI_H

#include <stdint.h>

#include "spmm_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spmm_multi* spmm_multi_t;

/* devices: ngpu device ordinals (NULL = 0 .. ngpu-1). Restores the caller's
 * current device before returning. RCCL is loaded here, at run time
 * (librccl.so.1): without it this returns SPMM_STATUS_NOT_INITIALIZED and
 * the rest of the library is unaffected. RCCL failures map to
 * SPMM_STATUS_EXECUTION_FAILED. */
spmm_status_t spmm_multi_create(spmm_multi_t* ctx, int ngpu, const int* devices);
spmm_status_t spmm_multi_destroy(spmm_multi_t ctx);
int spmm_multi_size(spmm_multi_t ctx);
/* Stream ordering with the caller for the NEXT spmm_csr_f32_multi call:
 * streams[p] is a hipStream_t on device p, a NULL entry being device p's
 * legacy null (default) stream; streams == NULL means no ordering. That
 * call first makes part p's compute stream wait for the work already queued
 * on streams[p] (the producers of B, the CSR arrays and C), and at the end
 * makes streams[p] wait for part p's last exchange, so work queued on
 * streams[p] afterwards sees all of C. The call then forgets the streams
 * (set them again before every call that needs the ordering), so no handle
 * is kept past the call it was given for. */
spmm_status_t spmm_multi_set_user_streams(spmm_multi_t ctx, void* const* streams);
/* The compute stream of part p (a hipStream_t; the call's results on device
 * p are complete once this stream is). */
spmm_status_t spmm_multi_get_stream(spmm_multi_t ctx, int part, void** stream);

/* Rows per chunk for a partition: ceil(max_p rows_p / chunks) (the same on
 * every part; a short part's trailing chunks are empty). */
int spmm_multi_slot_rows(int ngpu, const int* bounds, int chunks);

/* C = A(m x k, csr) * B(k x n), A row-partitioned by `bounds` (host,
 * ngpu + 1 entries, bounds[0] = 0, bounds[ngpu] = m).
 *   rowPtr[p], colInd[p], val[p]: device pointers on device p to part p's
 *     CSR: rowPtr[p] has rows_p + 1 entries and indexes colInd[p] / val[p]
 *     directly (it need not start at 0, so a view into the whole matrix's
 *     arrays uploaded to device p works);
 *   partNnz[p]: host, rowPtr[p][rows_p] - rowPtr[p][0] (sizes the grid);
 *   B[p]: device p's replica of B, row-major, ldb >= n;
 *   C[p]: device p's m x n output, row-major, ldc >= n (ldc == n when
 *     ngpu > 1).
 * Asynchronous on the parts' streams; spmm_multi_synchronize waits. Status
 * behaviour of spmm_csrmm_ex_f32 for bad sizes / pointers. */
spmm_status_t spmm_csr_f32_multi(spmm_multi_t ctx, int m, int n, int k, const int* bounds,
                                 const int* const* rowPtr, const int* const* colInd,
                                 const float* const* val, const int* partNnz,
                                 const float* const* B, int ldb, float* const* C, int ldc,
                                 int chunks);
spmm_status_t spmm_multi_synchronize(spmm_multi_t ctx);

/* Per-part timing of the last spmm_csr_f32_multi call (events on the
 * streams, recorded when enabled): compute_ms[p] = first kernel start to last
 * kernel end on device p, total_ms[p] = first kernel start to the end of
 * the last exchange on device p. Synchronises. */
spmm_status_t spmm_multi_set_timing(spmm_multi_t ctx, int enable);
spmm_status_t spmm_multi_get_times(spmm_multi_t ctx, float* compute_ms, float* total_ms);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SPMM_MULTI_H */
