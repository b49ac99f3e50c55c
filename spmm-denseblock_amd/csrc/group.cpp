// group.cpp — the group analyses of the grouped streams: bs 16 fp16
// (spmm_bsr16_group_analysis_f16 / spmm_bsrmm_grouped_f16) and bs 32 fp32
// (spmm_bsr32_group_analysis_f32 / spmm_bsrmm_grouped_f32), include/spmm_hip.h;
// DESIGN.md §4, "The grouped stream".
//
// Once per matrix, like spmm_bsr16_analysis_f16 and cuSPARSE's SpMM preprocess
// (the reference's rocsparse_bsrmm.h:102-256 has none), as two calls:
//  size query (buffer == NULL):
//  1. the device computes every block's column mask (bs 32: bsr32_analysis_kernel, masks
//     only; bs 16: grp_mask16_kernel in group_kernels.hip for 16-B aligned values);
//  2. grp_build_kernel PASS 1 (group_kernels.hip), one wave per group of W adjacent
//     block rows, checks the group's row pointer entries and block columns, merges
//     the W sorted block-column lists and counts the items of the union of their
//     nonzero columns in (block column J, column c) order, cut into items of E
//     entries (16 at bs 16, 8 at bs 32; the last one padded with row -1);
//  3. a one-workgroup scan sums the counts into the item pointers, a reduction
//     finds the largest block column and any bad group; 16 bytes come back to the
//     host (the analysis's one synchronisation) and size the buffer;
//  filling call (the caller's buffer, same arguments):
//  4. PASS 2 writes the B row J*bs + c of each entry and, per wave w of the group,
//     the block of row w holding (J, c) (-1: none, or that block's column c is all
//     zeros); grp_wmask_kernel then ORs the per-(item, wave) masks of the entries
//     whose source is a block (the MFMAs that wave runs at bs 32);
//  5. the fill kernels write each wave's A fragment of each item. At bs 32 the size
//     query's mask kernel (grp_mask32_kernel) also leaves a compact column-major copy of
//     ROW blocks' nonzero columns in a transient stream-ordered allocation (4 KB per
//     block, freed by the filling call), and the fill reads only those columns: one pass
//     over A instead of two (COLUMN blocks: the fill reads their columns in place).
// The filling call reuses the size query's device results (handle->grp_pending):
// the arrays must not change between the two calls, as between cuSPARSE's
// bufferSize and preprocess calls. It launches kernels and async copies only.
// Every size query recomputes those results, whatever ran before it.
// Round 4's first form merged on the host (0.27-0.46 s on the products stand-in),
// and its second ran the masks and PASS 1 again behind two synchronisations.
//
// Buffer layout (caller-owned device memory, bufferBytes from the first call):
//   [0, 256)                 header: word 0 = W, the block rows per group (the
//                            library's choice when groupRows was 0); the rest zero
//   item_ptr[ngroups + 1]    int32, the items of group g are [item_ptr[g], item_ptr[g+1])
//   rows[nitems][E]          int32, B row of each entry (-1: padding)
//   wmask[nitems][W]              uint32, bit e: entry e is a nonzero column of wave w's
//                                 block row (bs 32: the MFMAs it runs; bs 16: the B values
//                                 its fragments keep)
//   bs 16: afrag[nitems][W][128]  uint32, lane l of wave w: A[l & 15][4 (l >> 4) .. + 3] fp16 x 4
//   bs 32: afrag[nitems][W][32][8] fp32, A[row][entry] of wave w's block row
// The handle records the layout by buffer address (spmm_context::group_plans).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "context.hpp"

using namespace spmm;

namespace {

constexpr size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// The analysis of either stream: BS 16 (fp16 values, W = 2 / 4 / 8) or 32 (fp32, W = 2 / 4).
// Everything runs on the device. The size query (buffer == NULL): the column masks
// (bsr16 / bsr32_analysis_kernel, masks only), the per-group merge counting items
// (grp_build_kernel PASS 1, which also checks the row pointer), the item pointers'
// scan and the stats (largest block column, bad rows); one 16-B copy to the host
// and the only synchronisation of the analysis, for the size the caller must
// allocate. The results stay on the handle (grp_pending). The filling call
// (buffer != NULL) with the same arguments starts from them: the header and the
// item pointers into the buffer, the merge writing entries (PASS 2), the A
// fragments (the fill kernels); it neither synchronises nor reads anything on the
// host, so it can be captured in a graph. A filling call without that size query
// runs it first.
spmm_status_t group_analysis(spmm_handle_t handle, int BS, spmm_direction_t dir, int mb, int nnzb,
                             int groupRows, const int* bsrRowPtr, const int* bsrColInd,
                             const void* bsrVal, void* buffer, size_t* bufferBytes) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) || mb < 0 || nnzb < 0 ||
      !bufferBytes)
    return SPMM_STATUS_INVALID_VALUE;
  if (groupRows != 0 && groupRows != 2 && groupRows != 4 && (BS == 32 || groupRows != 8))
    return SPMM_STATUS_INVALID_VALUE;
  if (mb > 0 && !bsrRowPtr) return SPMM_STATUS_INVALID_VALUE;
  if (nnzb > 0 && (!bsrColInd || !bsrVal)) return SPMM_STATUS_INVALID_VALUE;
  // the mask and fill kernels read the values as f32x4 (BS 32) / u16x4 (BS 16)
  // vectors, as spmm_bsr32_analysis_f32 / spmm_bsr16_analysis_f16 require
  if (nnzb > 0 && reinterpret_cast<uintptr_t>(bsrVal) % (BS == 32 ? 16 : 8) != 0)
    return SPMM_STATUS_INVALID_VALUE;
  const int E = BS == 16 ? 16 : 8;  // entries per item
  hipStream_t st = handle->stream;
  std::lock_guard<std::mutex> glk(handle->grp_mu);  // the pending record, call to call
  auto& pend = handle->grp_pending;
  // Only a filling call reuses the pending size query, and only one of the same
  // arguments: a size query always runs, since the arrays at the same addresses may
  // hold another matrix by now (a caching allocator hands addresses out again).
  const bool same = buffer && pend.valid && pend.bs == BS && pend.req == groupRows &&
                    pend.dir == (int)dir && pend.mb == mb && pend.nnzb == nnzb &&
                    pend.rp == bsrRowPtr && pend.ci == bsrColInd && pend.val == bsrVal;
  if (!same) {
    // The size query. Candidates: groupRows itself, or at BS 16 with groupRows = 0 every W
    // (2, 4, 8), of which the one with the least modelled time is kept (below); BS 32 with 0
    // takes 2. grp_pend holds the masks [nnzb], per candidate the item pointers
    // [ngroups + 1], and per candidate 32 B of stats; the scratch the per-group counts and
    // largest block columns [2 ngroups] per candidate.
    pend.valid = false;
    int cand[3] = {groupRows, 0, 0}, nc = 1;
    if (groupRows == 0) {
      if (BS == 16) {
        cand[0] = 2;
        cand[1] = 4;
        cand[2] = 8;
        nc = 3;
      } else {
        cand[0] = 2;
      }
    }
    const size_t mk_bytes = align256((size_t)nnzb * 4);
    size_t ptr_off[3], cnt_off[3], stat_off = mk_bytes, scr = 0;
    for (int i = 0; i < nc; ++i) {
      const int ng = (mb + cand[i] - 1) / cand[i];
      ptr_off[i] = stat_off;
      stat_off = align256(stat_off + (size_t)(ng + 1) * 4);
      cnt_off[i] = scr;
      scr += align256((size_t)ng * 8);
    }
    if (spmm_status_t s = ensure_group_pending(handle, stat_off + 32 * nc)) return s;
    if (spmm_status_t s = ensure_scratch(handle, scr + 8)) return s;
    char* pb = static_cast<char*>(handle->grp_pend);
    unsigned* dmk = reinterpret_cast<unsigned*>(pb);
    hipError_t e = hipMemsetAsync(pb + stat_off, 0, 32 * nc, st);
    if (e != hipSuccess) return from_hip(e);
    // a previous size query's column copy (its filling call never came, or was captured)
    if (handle->grp_cols) {
      e = hipFreeAsync(handle->grp_cols, st);
      handle->grp_cols = nullptr;
      if (e != hipSuccess) return from_hip(e);
    }
    if (nnzb > 0 && mb > 0) {
      const auto* v16 = static_cast<const uint16_t*>(bsrVal);
      spmm_status_t s;
      if (BS == 32) {
        // ROW blocks: the compact column copy the fill reads, a 4-KB slot per block, when that
        // is at most kColsCap and a quarter of the free device memory (else, or without the
        // memory, the fill reads the blocks again: the RCM products stand-in's 10.5 M blocks
        // would take 43 GB for a copy of about 10)
        constexpr size_t kColsCap = size_t(16) << 30;
        const size_t want = (size_t)nnzb * 4096;
        size_t free_b = 0, total_b = 0;
        if (dir == SPMM_DIRECTION_ROW && want <= kColsCap &&
            hipMemGetInfo(&free_b, &total_b) == hipSuccess && want <= free_b / 4 &&
            hipMallocAsync(&handle->grp_cols, want, st) != hipSuccess) {
          (void)hipGetLastError();
          handle->grp_cols = nullptr;
        }
        s = launch_grp_mask32(handle, dir, nnzb, static_cast<const float*>(bsrVal), dmk,
                              static_cast<float*>(handle->grp_cols));
      } else {
        s = reinterpret_cast<uintptr_t>(bsrVal) % 16 == 0 ? launch_grp_mask16(handle, dir, nnzb, v16, dmk)
                                                          : launch_bsr16_analysis(handle, dir, nnzb, v16, dmk, nullptr);
      }
      if (s) return s;
    }
    for (int i = 0; i < nc; ++i) {
      const int ng = (mb + cand[i] - 1) / cand[i];
      int* dptr = reinterpret_cast<int*>(pb + ptr_off[i]);
      long long* dtot = reinterpret_cast<long long*>(pb + stat_off + 32 * i);
      int* dstat = reinterpret_cast<int*>(pb + stat_off + 32 * i + 8);
      int* dcnt = reinterpret_cast<int*>(static_cast<char*>(handle->scratch) + cnt_off[i]);
      int* dmaxj = dcnt + ng;
      if (mb > 0) {
        if (spmm_status_t s = launch_grp_build(handle, cand[i], BS, false, mb, nnzb, ng, bsrRowPtr,
                                               bsrColInd, dmk, dcnt, dmaxj, nullptr, nullptr,
                                               nullptr))
          return s;
        if (spmm_status_t s = launch_scan_counts(handle, dcnt, ng, dptr, dtot)) return s;
        if (spmm_status_t s = launch_grp_stats(handle, dmaxj, ng, dstat)) return s;
      } else {
        e = hipMemsetAsync(dptr, 0, 4, st);
        if (e == hipSuccess) e = hipMemsetAsync(dstat, 0xff, 4, st);  // max_col -1
        if (e != hipSuccess) return from_hip(e);
      }
    }
    struct Stat { long long total; int max_col, bad, pad[4]; } host[3]{};
    static_assert(sizeof(Stat) == 32, "stats record");
    e = hipMemcpyAsync(host, pb + stat_off, 32 * nc, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return from_hip(e);
    if (host[0].bad) return SPMM_STATUS_INVALID_VALUE;  // a bad row pointer or negative block column
    // The choice at BS 16: modelled time items(W) * (kCopy + W) per column tile. An item
    // costs its 16 B-row copies and barrier once per workgroup (kCopy, in units of one
    // wave's 16 MFMAs and transposed reads of the item) plus W waves' MFMAs, every wave
    // multiplying every item whether its block row holds the entries or not. kCopy = 2.74
    // fits round 4's products stand-in (1.39 M items at W = 2, 0.88 M at W = 4: 3.19
    // against 2.87 ms); it picks W = 2 where the rows share few columns (a union about
    // the sum of the rows') and W = 4 or 8 where they share many.
    int pick = 0;
    if (nc > 1) {
      constexpr double kCopy = 2.74;
      double best = -1.0;
      for (int i = 0; i < nc; ++i) {
        const double t = (double)host[i].total * (kCopy + cand[i]);
        if (best < 0.0 || t < best) {
          best = t;
          pick = i;
        }
      }
    }
    const int W = cand[pick];
    const int ngroups = (mb + W - 1) / W;
    if (host[pick].total > INT_MAX) return SPMM_STATUS_NOT_SUPPORTED;  // int32 item pointers
    const long long nitems = host[pick].total;
    pend.rows_off = align256(256 + (size_t)(ngroups + 1) * 4);
    pend.wmask_off = align256(pend.rows_off + (size_t)nitems * E * 4);
    pend.afrag_off = align256(pend.wmask_off + (size_t)nitems * W * 4);
    pend.need = pend.afrag_off + (size_t)nitems * W * (BS == 16 ? 512 : 1024);
    pend.nitems = nitems;
    pend.max_col = host[pick].max_col;
    pend.ptr_off = ptr_off[pick];
    pend.bs = BS;
    pend.W = W;
    pend.req = groupRows;
    pend.dir = (int)dir;
    pend.mb = mb;
    pend.nnzb = nnzb;
    pend.rp = bsrRowPtr;
    pend.ci = bsrColInd;
    pend.val = bsrVal;
    pend.valid = true;
  }
  const int W = pend.W;
  const int ngroups = (mb + W - 1) / W;
  if (!buffer) {
    *bufferBytes = pend.need;
    return SPMM_STATUS_SUCCESS;
  }
  if (*bufferBytes < pend.need) return SPMM_STATUS_INVALID_VALUE;
  pend.valid = false;  // consumed: another analysis starts from its own size query
  const long long nitems = pend.nitems;
  char* buf = static_cast<char*>(buffer);
  const char* pb = static_cast<const char*>(handle->grp_pend);
  hipError_t e = hipMemsetAsync(buf, 0, 256, st);
  if (e == hipSuccess) e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(buf), W, 1, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(buf + 256, pb + pend.ptr_off, (size_t)(ngroups + 1) * 4,
                       hipMemcpyDeviceToDevice, st);
  // the alignment gaps between the sections are zeroed, so the buffer's bytes are a
  // function of the matrix alone (an analysis compares byte for byte with another)
  const size_t gaps[3][2] = {{256 + (size_t)(ngroups + 1) * 4, pend.rows_off},
                             {pend.rows_off + (size_t)nitems * E * 4, pend.wmask_off},
                             {pend.wmask_off + (size_t)nitems * W * 4, pend.afrag_off}};
  for (const auto& g : gaps)
    if (e == hipSuccess && g[1] > g[0]) e = hipMemsetAsync(buf + g[0], 0, g[1] - g[0], st);
  if (e != hipSuccess) return from_hip(e);
  if (nitems) {
    // the entry sources in the workspace (the masks stay in grp_pend)
    if (spmm_status_t s = ensure_workspace(handle, (size_t)nitems * E * W * 4)) return s;
    int* dsrc = static_cast<int*>(handle->ws);
    int* drows = reinterpret_cast<int*>(buf + pend.rows_off);
    if (spmm_status_t s = launch_grp_build(handle, W, BS, true, mb, nnzb, ngroups, bsrRowPtr,
                                           bsrColInd, reinterpret_cast<const unsigned*>(pb), nullptr,
                                           nullptr, reinterpret_cast<const int*>(buf + 256), drows,
                                           dsrc))
      return s;
    if (spmm_status_t s = launch_grp_wmask(handle, nitems, W, E, dsrc,
                                           reinterpret_cast<unsigned*>(buf + pend.wmask_off)))
      return s;
    float* afrag = reinterpret_cast<float*>(buf + pend.afrag_off);
    // a captured fill reads the values themselves: a graph replayed later must not read the
    // transient column copy, which the next size query frees
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing =
        hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
    spmm_status_t s;
    if (BS == 16)
      s = launch_bsr16_grp_fill(handle, nitems, W, dir, drows, dsrc,
                                static_cast<const uint16_t*>(bsrVal),
                                reinterpret_cast<unsigned*>(afrag));
    else if (dir == SPMM_DIRECTION_COLUMN)  // a column of a COLUMN block is contiguous
      s = launch_bsr32_grp_fillc(handle, nitems, W, drows, dsrc, static_cast<const float*>(bsrVal),
                                 nullptr, afrag);
    else if (handle->grp_cols && !capturing)
      s = launch_bsr32_grp_fillc(handle, nitems, W, drows, dsrc,
                                 static_cast<const float*>(handle->grp_cols),
                                 reinterpret_cast<const unsigned*>(pb), afrag);
    else
      s = launch_bsr32_grp_fill(handle, nitems, W, dir, drows, dsrc,
                                static_cast<const float*>(bsrVal), afrag);
    if (s) return s;
  }
  // the column copy is spent; under stream capture it stays for the next size query (or
  // spmm_destroy) to free, the free being no node of the caller's graph
  if (handle->grp_cols && BS == 32) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
      hipError_t fe = hipFreeAsync(handle->grp_cols, st);
      handle->grp_cols = nullptr;
      if (fe != hipSuccess) return from_hip(fe);
    }
  }
  std::lock_guard<std::mutex> lk(handle->mu);
  spmm_context::GroupPlan plan{W, mb, ngroups, nitems, pend.need, pend.rows_off, pend.afrag_off,
                               pend.max_col};
  plan.bs = BS;
  plan.wmask_off = pend.wmask_off;
  handle->group_plans[buffer] = plan;
  return SPMM_STATUS_SUCCESS;
}

// The plan of `buffer` for a product at block size BS, or an error status.
spmm_status_t find_plan(spmm_handle_t handle, const void* buffer, int BS, int mb, int kb,
                        spmm_context::GroupPlan* plan) {
  std::lock_guard<std::mutex> lk(handle->mu);
  auto it = handle->group_plans.find(buffer);
  if (it == handle->group_plans.end() || it->second.bs != BS) return SPMM_STATUS_INVALID_VALUE;
  *plan = it->second;
  if (plan->mb != mb || plan->max_col >= kb) return SPMM_STATUS_INVALID_VALUE;
  return SPMM_STATUS_SUCCESS;
}

}  // namespace

extern "C" {

spmm_status_t spmm_bsr16_group_analysis_f16(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                            int nnzb, int groupRows, const int* bsrRowPtr,
                                            const int* bsrColInd, const uint16_t* bsrVal,
                                            void* buffer, size_t* bufferBytes) {
  return group_analysis(handle, 16, dir, mb, nnzb, groupRows, bsrRowPtr, bsrColInd, bsrVal, buffer,
                        bufferBytes);
}

spmm_status_t spmm_bsr32_group_analysis_f32(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                            int nnzb, int groupRows, const int* bsrRowPtr,
                                            const int* bsrColInd, const float* bsrVal,
                                            void* buffer, size_t* bufferBytes) {
  return group_analysis(handle, 32, dir, mb, nnzb, groupRows, bsrRowPtr, bsrColInd, bsrVal, buffer,
                        bufferBytes);
}

spmm_status_t spmm_bsrmm_grouped_f16(spmm_handle_t handle, int mb, int kb, int n,
                                     const void* buffer, float alpha, const uint16_t* B, int ldb,
                                     spmm_order_t orderB, float beta, float* C, int ldc,
                                     spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (mb < 0 || kb < 0 || n < 0) return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (mb == 0 || n == 0 || kb == 0) return SPMM_STATUS_SUCCESS;
  if (!buffer || !B || !C) return SPMM_STATUS_INVALID_VALUE;
  spmm_context::GroupPlan plan;
  if (spmm_status_t st = find_plan(handle, buffer, 16, mb, kb, &plan)) return st;
  const long long K = (long long)kb * 16, M = (long long)mb * 16;
  if (orderB == SPMM_ORDER_COL ? ldb < K : ldb < n) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_COL ? ldc < M : ldc < n) return SPMM_STATUS_INVALID_VALUE;
  // the stream copies whole 16-B chunks of 256-column B-row pieces
  if (n < 8 || n % 8 || reinterpret_cast<uintptr_t>(B) % 16) return SPMM_STATUS_NOT_SUPPORTED;
  const char* buf = static_cast<const char*>(buffer);
  const uint16_t* Bx = B;
  int ldbx = ldb;
  if (orderB == SPMM_ORDER_COL) {  // staged row-major in the workspace, as the column streams
    if (spmm_status_t s = ensure_workspace(handle, (size_t)K * n * 2)) return s;
    uint16_t* Bt = static_cast<uint16_t*>(handle->ws);
    if (spmm_status_t s = launch_transpose16(handle, n, (int)K, B, ldb, Bt, n)) return s;
    Bx = Bt;
    ldbx = n;
  } else if (ldb % 8) {
    return SPMM_STATUS_NOT_SUPPORTED;
  }
  return launch_bsrmm_grouped_f16(
      handle, plan.W, mb, n, plan.ngroups, reinterpret_cast<const int*>(buf + 256),
      reinterpret_cast<const int*>(buf + plan.rows_off),
      reinterpret_cast<const unsigned*>(buf + plan.wmask_off),
      reinterpret_cast<const unsigned*>(buf + plan.afrag_off), Bx, ldbx, alpha, beta, C, ldc,
      orderC == SPMM_ORDER_ROW);
}

spmm_status_t spmm_bsrmm_grouped_f32(spmm_handle_t handle, int mb, int kb, int n,
                                     const void* buffer, float alpha, const float* B, int ldb,
                                     spmm_order_t orderB, float beta, float* C, int ldc,
                                     spmm_order_t orderC) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (mb < 0 || kb < 0 || n < 0) return SPMM_STATUS_INVALID_VALUE;
  if ((orderB != SPMM_ORDER_ROW && orderB != SPMM_ORDER_COL) ||
      (orderC != SPMM_ORDER_ROW && orderC != SPMM_ORDER_COL))
    return SPMM_STATUS_INVALID_VALUE;
  if (mb == 0 || n == 0 || kb == 0) return SPMM_STATUS_SUCCESS;
  if (!buffer || !B || !C) return SPMM_STATUS_INVALID_VALUE;
  spmm_context::GroupPlan plan;
  if (spmm_status_t st = find_plan(handle, buffer, 32, mb, kb, &plan)) return st;
  const long long K = (long long)kb * 32, M = (long long)mb * 32;
  if (orderB == SPMM_ORDER_COL ? ldb < K : ldb < n) return SPMM_STATUS_INVALID_VALUE;
  if (orderC == SPMM_ORDER_COL ? ldc < M : ldc < n) return SPMM_STATUS_INVALID_VALUE;
  // the stream copies 16-B pieces of 128-column B-row tiles and stores 16-B pieces of C rows
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (n % 4 || !al16(B) || !al16(C)) return SPMM_STATUS_NOT_SUPPORTED;
  if ((orderB == SPMM_ORDER_ROW && ldb % 4) || (orderC == SPMM_ORDER_ROW && ldc % 4))
    return SPMM_STATUS_NOT_SUPPORTED;
  // column-major B / C are staged row-major in the workspace (B first, then C)
  const size_t bbytes = orderB == SPMM_ORDER_COL ? (size_t)K * n * 4 : 0;
  const size_t cbytes = orderC == SPMM_ORDER_COL ? (size_t)M * n * 4 : 0;
  if (bbytes + cbytes)
    if (spmm_status_t s = ensure_workspace(handle, bbytes + cbytes)) return s;
  const float* Bx = B;
  int ldbx = ldb;
  if (bbytes) {
    float* Bt = static_cast<float*>(handle->ws);
    if (spmm_status_t s = launch_transpose(handle, n, (int)K, B, ldb, Bt, n, 0.f)) return s;
    Bx = Bt;
    ldbx = n;
  }
  const char* buf = static_cast<const char*>(buffer);
  float* Cx = C;
  int ldcx = ldc;
  float bx = beta;
  if (cbytes) {  // alpha A B into a row-major tile, then C = tile^T + beta C
    Cx = reinterpret_cast<float*>(static_cast<char*>(handle->ws) + bbytes);
    ldcx = n;
    bx = 0.f;
  }
  if (spmm_status_t s = launch_bsrmm_grouped_f32(
          handle, plan.W, mb, n, plan.ngroups, reinterpret_cast<const int*>(buf + 256),
          reinterpret_cast<const int*>(buf + plan.rows_off),
          reinterpret_cast<const unsigned*>(buf + plan.wmask_off),
          reinterpret_cast<const float*>(buf + plan.afrag_off), Bx, ldbx, alpha, bx, Cx, ldcx))
    return s;
  if (cbytes) return launch_transpose(handle, (int)M, n, Cx, ldcx, C, ldc, beta);
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_bsr16_group_release(spmm_handle_t handle, const void* buffer) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  std::lock_guard<std::mutex> lk(handle->mu);
  handle->group_plans.erase(buffer);
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_bsr_group_release(spmm_handle_t handle, const void* buffer) {
  return spmm_bsr16_group_release(handle, buffer);
}

}  // extern "C"
