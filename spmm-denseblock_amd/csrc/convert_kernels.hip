// convert_kernels.hip — CSR <-> BSR conversion on the device (SURVEY.md §8f
// rank 4): the device-pointer forms of cusparseXcsr2bsrNnz / cusparseScsr2bsr
// (run_bsrmm.cu:116-142) and cusparseSbsr2csr (bsr2csr.cu:186-188).
//
// csr2bsr: one wave per block row merges the block row's bs sorted CSR rows
// (lane l holds row l's cursor; bs <= 64): each step takes the wave minimum
// of the lanes' head block columns, and every lane whose head is that block
// column consumes all its entries in it. Pass 1 counts the distinct block
// columns, a single-workgroup scan turns the counts into bsrRowPtr, pass 2
// writes the block columns and scatters the values into the zero-filled
// blocks. Duplicate entries (same row and column) are summed in CSR order by
// the lane that owns the row, so the result is bit-identical to the host
// conversion (spmm_scsr2bsr). Rows must be sorted by column, as cuSPARSE
// requires for its csrSorted* arguments.
//
// bsr2csr: every block row expands to bs CSR rows of equal length
// (blocks * bs), so the row pointer has a closed form and each wave writes
// its block row's entries with coalesced stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "context.hpp"

namespace {

constexpr int kWave = 64;
constexpr int kWG = 256;

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// Cursor of one CSR row inside a block row (lane-private).
struct RowCursor {
  int ptr, end, bs, n;
  const int* colind;
  int base;
  __device__ __forceinline__ int col(int p) const { return colind[p] - base; }
  // Block column of the head entry; INT_MAX when the row is exhausted.
  // Entries with a column outside [0, n) are skipped (and flagged).
  __device__ __forceinline__ int head(int* bad) {
    while (ptr < end) {
      const int c = col(ptr);
      if (c >= 0 && c < n) return c / bs;
      *bad = 1;
      ++ptr;
    }
    return INT_MAX;
  }
};

template <bool FILL, bool ROWDIR>
__global__ __launch_bounds__(kWG) void csr2bsr_kernel(int m, int n, int mb, int bs,
                                                      const int* __restrict__ rowptr,
                                                      const int* __restrict__ colind,
                                                      const float* __restrict__ val, int baseA,
                                                      int* __restrict__ count,
                                                      const int* __restrict__ bsr_rowptr,
                                                      int baseC, int* __restrict__ bsr_colind,
                                                      float* __restrict__ bsr_val,
                                                      int* __restrict__ bad) {
  const int lane = threadIdx.x & (kWave - 1);
  const int br = blockIdx.x * (kWG / kWave) + (threadIdx.x >> 6);
  if (br >= mb) return;
  const int r = br * bs + lane;
  RowCursor cur{0, 0, bs, n, colind, baseA};
  if (lane < bs && r < m) {
    cur.ptr = rowptr[r] - baseA;
    cur.end = rowptr[r + 1] - baseA;
  }
  int flag = 0;
  int hd = cur.head(&flag);
  const size_t bs2 = (size_t)bs * bs;
  int k = FILL ? bsr_rowptr[br] - baseC : 0;
  int t = 0;
  while (true) {
    const int mn = wave_min(hd);
    if (mn == INT_MAX) break;
    if (FILL && lane == 0) bsr_colind[k] = mn + baseC;
    if (hd == mn) {
      int prev = -1;
      while (cur.ptr < cur.end) {
        const int c = cur.col(cur.ptr);
        if (c < 0 || c >= n) {  // skipped, as in head()
          flag = 1;
          ++cur.ptr;
          continue;
        }
        if (c / bs != mn) break;
        if constexpr (FILL) {
          const int cc = c % bs;
          float* p = bsr_val + (size_t)k * bs2 +
                     (ROWDIR ? (size_t)lane * bs + cc : (size_t)cc * bs + lane);
          const float v = val[cur.ptr];
          *p = (c == prev) ? *p + v : v;  // duplicates summed in CSR order
        }
        prev = c;
        ++cur.ptr;
      }
      hd = cur.head(&flag);
    }
    ++k;
    ++t;
  }
  if (!FILL && lane == 0) count[br] = t;
  if (flag) *bad = 1;
}

// Exclusive scan of count[0..mb) into out[0..mb] (+ base), one workgroup: each thread sums
// kScanPer consecutive counts, the workgroup scans the sums, and each thread writes its
// counts' prefixes (16 K counts per pass; one count per thread took 63 us on 76 K counts).
constexpr int kScanPer = 16;

__global__ __launch_bounds__(1024) void scan_kernel(const int* __restrict__ count, int mb,
                                                    int base, int* __restrict__ out,
                                                    long long* __restrict__ total) {
  __shared__ long long part[1024 / kWave];
  __shared__ long long carry;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (long long c0 = 0; c0 < mb; c0 += 1024 * kScanPer) {
    const long long i0 = c0 + (long long)tid * kScanPer;
    int v[kScanPer];
    long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = i0 + k < mb ? count[i0 + k] : 0;
      s += v[k];
    }
    // inclusive wave scan of the threads' sums
    long long x = s;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const long long y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == kWave - 1) part[wv] = x;
    __syncthreads();
    long long off = carry;
    for (int w = 0; w < wv; ++w) off += part[w];
    long long run = off + x - s;  // before this thread's first count
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      run += v[k];
      if (i0 + k < mb) out[i0 + k + 1] = (int)(run + base);
    }
    __syncthreads();
    if (tid == 1023) carry = off + x;
    __syncthreads();
  }
  if (tid == 0) {
    out[0] = base;
    *total = carry;
  }
}

template <bool ROWDIR>
__global__ __launch_bounds__(kWG) void bsr2csr_kernel(int mb, int bs,
                                                      const int* __restrict__ bsr_rowptr,
                                                      const int* __restrict__ bsr_colind,
                                                      const float* __restrict__ bsr_val,
                                                      int baseA, int baseC,
                                                      int* __restrict__ csr_rowptr,
                                                      int* __restrict__ csr_colind,
                                                      float* __restrict__ csr_val) {
  const int lane = threadIdx.x & (kWave - 1);
  const int br = blockIdx.x * (kWG / kWave) + (threadIdx.x >> 6);
  if (br >= mb) return;
  const int k0 = bsr_rowptr[br] - baseA, k1 = bsr_rowptr[br + 1] - baseA;
  const long long bs2 = (long long)bs * bs;
  const int len = (k1 - k0) * bs;  // entries per CSR row of this block row
  for (int rr = lane; rr < bs; rr += kWave)
    csr_rowptr[(size_t)br * bs + rr] = (int)(k0 * bs2 + (long long)rr * len) + baseC;
  if (br == mb - 1 && lane == 0)
    csr_rowptr[(size_t)mb * bs] = (int)(k1 * bs2) + baseC;
  for (int rr = 0; rr < bs; ++rr) {
    const size_t rstart = (size_t)(k0 * bs2 + (long long)rr * len);
    for (int e = lane; e < len; e += kWave) {
      const int k = k0 + e / bs, c = e % bs;
      csr_colind[rstart + e] = (bsr_colind[k] - baseA) * bs + c + baseC;
      csr_val[rstart + e] = bsr_val[(size_t)k * bs2 + (ROWDIR ? (size_t)rr * bs + c
                                                              : (size_t)c * bs + rr)];
    }
  }
}

// coo2csr (cusparseXcoo2csr, csrmm.cu:148-149): row pointer of a row-sorted
// COO. Thread r writes csr_rowptr[r] = (first entry with row >= r) + base by
// a binary search over the sorted row indices; O(m log nnz), no atomics, so
// it is exact and deterministic for any row distribution (empty rows,
// power-law hubs).
__global__ __launch_bounds__(256) void coo2csr_kernel(const int* __restrict__ coo_row, int nnz,
                                                      int m, int base,
                                                      int* __restrict__ csr_rowptr) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > m) return;
  int lo = 0, hi = nnz;  // first index with coo_row[i] - base >= r
  while (lo < hi) {
    const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
    if (coo_row[mid] - base < r) lo = mid + 1;
    else hi = mid;
  }
  csr_rowptr[r] = lo + base;
}

// Re-blocking to bs 32 (spmm_xbsr_reblock32_nnzb / spmm_sbsr_reblock32): a small
// block (bs = 2 / 4 / 8 / 16, R = 32 / bs of them per side of a 32 x 32 block) of
// block row I and block column J lies inside the 32 x 32 block (I / R, J / R), at
// sub-block (I % R, J % R). One wave per 32-row block row merges its R block rows'
// sorted block-column lists on J / R (lane r < R holds block row I32 * R + r's
// cursor): PASS 1 counts the distinct J / R, PASS 2 writes them and, per small
// block, its 32 x 32 block and the element offset of its sub-block there.
template <bool FILL>
__global__ __launch_bounds__(kWG) void reblock32_kernel(int mb, int R, int shift,
                                                        const int* __restrict__ rowptr,
                                                        const int* __restrict__ colind,
                                                        int* __restrict__ count,
                                                        const int* __restrict__ rowptr32,
                                                        int* __restrict__ colind32,
                                                        int* __restrict__ map_k,
                                                        int* __restrict__ map_off, int bs,
                                                        int rowdir, int* __restrict__ bad) {
  const int lane = threadIdx.x & (kWave - 1);
  const int mb32 = (mb + R - 1) / R;
  const int br = blockIdx.x * (kWG / kWave) + (threadIdx.x >> 6);
  if (br >= mb32) return;
  const int I = br * R + lane;
  int ptr = 0, end = 0;
  if (lane < R && I < mb) {
    ptr = rowptr[I];
    end = rowptr[I + 1];
  }
  int flag = 0;
  auto head = [&]() -> int {
    while (ptr < end) {
      const int J = colind[ptr];
      if (J >= 0) return J >> shift;
      flag = 1;  // a negative block column: skipped and reported
      ++ptr;
    }
    return INT_MAX;
  };
  int hd = head();
  int k = FILL ? rowptr32[br] : 0;
  int t = 0;
  while (true) {
    const int mn = wave_min(hd);
    if (mn == INT_MAX) break;
    if (FILL && lane == 0) colind32[k] = mn;
    if (hd == mn) {
      while (ptr < end) {
        const int J = colind[ptr];
        if (J < 0) {
          flag = 1;
          ++ptr;
          continue;
        }
        if ((J >> shift) != mn) break;
        if constexpr (FILL) {
          const int sc = (J & (R - 1)) * bs, sr = lane * bs;  // sub-block column / row
          map_k[ptr] = k;
          map_off[ptr] = rowdir ? sr * 32 + sc : sc * 32 + sr;
        }
        ++ptr;
      }
      hd = head();
    }
    ++k;
    ++t;
  }
  if (!FILL && lane == 0) count[br] = t;
  if (flag) *bad = 1;
}

// Element e of small block b to its place in the zero-filled bs 32 values (ROW: e =
// row * bs + col, COLUMN: e = col * bs + row; both land at off + (e / bs) * 32 + e % bs).
__global__ __launch_bounds__(256) void reblock32_values_kernel(long long total, int bs, int bs2,
                                                               const float* __restrict__ val,
                                                               const int* __restrict__ map_k,
                                                               const int* __restrict__ map_off,
                                                               float* __restrict__ val32) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / bs2;
    const int e = (int)(i - b * bs2);
    val32[(size_t)map_k[b] * 1024 + map_off[b] + (e / bs) * 32 + e % bs] = val[i];
  }
}

}  // namespace

namespace spmm {

spmm_status_t launch_scan_counts(spmm_context* ctx, const int* count, int n, int* out,
                                 long long* total) {
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, count, n, 0, out, total);
  return from_hip(hipGetLastError());
}

}  // namespace spmm

extern "C" {

spmm_status_t spmm_xcoo2csr(spmm_handle_t handle, const int* cooRowInd, int nnz, int m,
                            int* csrRowPtr, spmm_index_base_t idxBase) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (nnz < 0 || m < 0 || (idxBase != SPMM_INDEX_BASE_ZERO && idxBase != SPMM_INDEX_BASE_ONE))
    return SPMM_STATUS_INVALID_VALUE;
  if (!csrRowPtr || (nnz > 0 && !cooRowInd)) return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = handle;
  hipLaunchKernelGGL(coo2csr_kernel, dim3((m + 1 + 255) / 256), dim3(256), 0, ctx->stream,
                     cooRowInd, nnz, m, (int)idxBase, csrRowPtr);
  return spmm::from_hip(hipGetLastError());
}

spmm_status_t spmm_xcsr2bsr_nnz_dev(spmm_handle_t handle, spmm_direction_t dir, int m, int n,
                                    const spmm_mat_descr_t descrA, const int* csrRowPtr,
                                    const int* csrColInd, int blockDim,
                                    const spmm_mat_descr_t descrC, int* bsrRowPtr,
                                    int* nnzTotalHostPtr) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (!descrA || !descrC || m < 0 || n < 0 || blockDim <= 0 || blockDim > kWave)
    return SPMM_STATUS_INVALID_VALUE;
  if (!csrRowPtr || !bsrRowPtr || !nnzTotalHostPtr) return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = handle;
  const int mb = (m + blockDim - 1) / blockDim;
  // workspace: counts [mb] + total (8 B) + error flag
  const size_t need = sizeof(int) * (size_t)mb + 16 + 16;
  if (spmm_status_t st = spmm::ensure_workspace(ctx, need); st != SPMM_STATUS_SUCCESS) return st;
  char* ws = static_cast<char*>(ctx->ws);
  long long* total = reinterpret_cast<long long*>(ws);
  int* bad = reinterpret_cast<int*>(ws + 8);
  int* count = reinterpret_cast<int*>(ws + 32);
  if (hipMemsetAsync(ws, 0, 32, ctx->stream) != hipSuccess) return SPMM_STATUS_EXECUTION_FAILED;
  if (mb > 0)
    hipLaunchKernelGGL((csr2bsr_kernel<false, true>), dim3((mb + 3) / 4), dim3(kWG), 0,
                       ctx->stream, m, n, mb, blockDim, csrRowPtr, csrColInd, nullptr,
                       (int)descrA->base, count, nullptr, 0, nullptr, nullptr, bad);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, count, mb,
                     (int)descrC->base, bsrRowPtr, total);
  long long host[2] = {0, 0};
  if (hipMemcpyAsync(host, ws, 16, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return SPMM_STATUS_EXECUTION_FAILED;
  if ((int)(host[1] & 0xffffffff) != 0) return SPMM_STATUS_INVALID_VALUE;  // bad column
  if (host[0] > INT32_MAX) return SPMM_STATUS_INVALID_VALUE;
  *nnzTotalHostPtr = (int)host[0];
  return spmm::from_hip(hipGetLastError());
}

spmm_status_t spmm_scsr2bsr_dev(spmm_handle_t handle, spmm_direction_t dir, int m, int n,
                                const spmm_mat_descr_t descrA, const float* csrVal,
                                const int* csrRowPtr, const int* csrColInd, int blockDim,
                                const spmm_mat_descr_t descrC, float* bsrVal,
                                const int* bsrRowPtr, int* bsrColInd) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (!descrA || !descrC || m < 0 || n < 0 || blockDim <= 0 || blockDim > kWave)
    return SPMM_STATUS_INVALID_VALUE;
  if (!csrRowPtr || !bsrRowPtr || !csrColInd || !csrVal || !bsrColInd || !bsrVal)
    return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = handle;
  const int mb = (m + blockDim - 1) / blockDim;
  if (mb == 0) return SPMM_STATUS_SUCCESS;
  int last[2];  // nnzb from the row pointer (device), for the zero fill
  if (hipMemcpyAsync(last, bsrRowPtr, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) !=
          hipSuccess ||
      hipMemcpyAsync(last + 1, bsrRowPtr + mb, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) !=
          hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return SPMM_STATUS_EXECUTION_FAILED;
  const long long nnzb = (long long)last[1] - last[0];
  if (nnzb < 0) return SPMM_STATUS_INVALID_VALUE;
  if (spmm_status_t st = spmm::ensure_workspace(ctx, 16); st != SPMM_STATUS_SUCCESS) return st;
  int* bad = static_cast<int*>(ctx->ws);
  if (hipMemsetAsync(bad, 0, sizeof(int), ctx->stream) != hipSuccess ||
      (nnzb > 0 && hipMemsetAsync(bsrVal, 0, sizeof(float) * (size_t)nnzb * blockDim * blockDim,
                                  ctx->stream) != hipSuccess))
    return SPMM_STATUS_EXECUTION_FAILED;
  const dim3 grid((mb + 3) / 4);
  if (dir == SPMM_DIRECTION_ROW)
    hipLaunchKernelGGL((csr2bsr_kernel<true, true>), grid, dim3(kWG), 0, ctx->stream, m, n, mb,
                       blockDim, csrRowPtr, csrColInd, csrVal, (int)descrA->base, nullptr,
                       bsrRowPtr, (int)descrC->base, bsrColInd, bsrVal, bad);
  else
    hipLaunchKernelGGL((csr2bsr_kernel<true, false>), grid, dim3(kWG), 0, ctx->stream, m, n, mb,
                       blockDim, csrRowPtr, csrColInd, csrVal, (int)descrA->base, nullptr,
                       bsrRowPtr, (int)descrC->base, bsrColInd, bsrVal, bad);
  return spmm::from_hip(hipGetLastError());
}

spmm_status_t spmm_sbsr2csr_dev(spmm_handle_t handle, spmm_direction_t dir, int mb, int nb,
                                const spmm_mat_descr_t descrA, const float* bsrVal,
                                const int* bsrRowPtr, const int* bsrColInd, int blockDim,
                                const spmm_mat_descr_t descrC, float* csrVal, int* csrRowPtr,
                                int* csrColInd) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (!descrA || !descrC || mb < 0 || nb < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!bsrRowPtr || !csrRowPtr) return SPMM_STATUS_INVALID_VALUE;
  (void)nb;
  spmm_context* ctx = handle;
  if (mb == 0) return SPMM_STATUS_SUCCESS;
  const dim3 grid((mb + 3) / 4);
  if (dir == SPMM_DIRECTION_ROW)
    hipLaunchKernelGGL((bsr2csr_kernel<true>), grid, dim3(kWG), 0, ctx->stream, mb, blockDim,
                       bsrRowPtr, bsrColInd, bsrVal, (int)descrA->base, (int)descrC->base,
                       csrRowPtr, csrColInd, csrVal);
  else
    hipLaunchKernelGGL((bsr2csr_kernel<false>), grid, dim3(kWG), 0, ctx->stream, mb, blockDim,
                       bsrRowPtr, bsrColInd, bsrVal, (int)descrA->base, (int)descrC->base,
                       csrRowPtr, csrColInd, csrVal);
  return spmm::from_hip(hipGetLastError());
}

spmm_status_t spmm_xbsr_reblock32_nnzb(spmm_handle_t handle, spmm_direction_t dir, int mb,
                                       int nnzb, int blockDim, const int* bsrRowPtr,
                                       const int* bsrColInd, int* bsrRowPtr32,
                                       int* nnzb32HostPtr) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) || mb < 0 || nnzb < 0 ||
      !nnzb32HostPtr)
    return SPMM_STATUS_INVALID_VALUE;
  if (blockDim != 2 && blockDim != 4 && blockDim != 8 && blockDim != 16 && blockDim != 32)
    return SPMM_STATUS_INVALID_VALUE;
  if (!bsrRowPtr32 || (mb > 0 && !bsrRowPtr) || (nnzb > 0 && !bsrColInd))
    return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = handle;
  const int R = 32 / blockDim, shift = __builtin_ctz(R);
  const int mb32 = (mb + R - 1) / R;
  const size_t need = 32 + (((size_t)mb32 * 4 + 255) & ~(size_t)255);
  if (spmm_status_t st = spmm::ensure_workspace(ctx, need); st != SPMM_STATUS_SUCCESS) return st;
  char* ws = static_cast<char*>(ctx->ws);
  long long* total = reinterpret_cast<long long*>(ws);
  int* bad = reinterpret_cast<int*>(ws + 8);
  int* count = reinterpret_cast<int*>(ws + 32);
  if (hipMemsetAsync(ws, 0, 32, ctx->stream) != hipSuccess) return SPMM_STATUS_EXECUTION_FAILED;
  if (mb32 > 0)
    hipLaunchKernelGGL(reblock32_kernel<false>, dim3((mb32 + 3) / 4), dim3(kWG), 0, ctx->stream,
                       mb, R, shift, bsrRowPtr, bsrColInd, count, nullptr, nullptr, nullptr,
                       nullptr, blockDim, dir == SPMM_DIRECTION_ROW ? 1 : 0, bad);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, count, mb32, 0,
                     bsrRowPtr32, total);
  long long host[2] = {0, 0};
  if (hipMemcpyAsync(host, ws, 16, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return SPMM_STATUS_EXECUTION_FAILED;
  if ((int)(host[1] & 0xffffffff) != 0) return SPMM_STATUS_INVALID_VALUE;  // negative column
  if (host[0] > INT32_MAX) return SPMM_STATUS_NOT_SUPPORTED;
  *nnzb32HostPtr = (int)host[0];
  return spmm::from_hip(hipGetLastError());
}

spmm_status_t spmm_sbsr_reblock32(spmm_handle_t handle, spmm_direction_t dir, int mb, int nnzb,
                                  int blockDim, const int* bsrRowPtr, const int* bsrColInd,
                                  const float* bsrVal, const int* bsrRowPtr32, int nnzb32,
                                  int* bsrColInd32, float* bsrVal32) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if ((dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) || mb < 0 || nnzb < 0 ||
      nnzb32 < 0)
    return SPMM_STATUS_INVALID_VALUE;
  if (blockDim != 2 && blockDim != 4 && blockDim != 8 && blockDim != 16 && blockDim != 32)
    return SPMM_STATUS_INVALID_VALUE;
  if (!bsrRowPtr32 || (mb > 0 && !bsrRowPtr) || (nnzb > 0 && (!bsrColInd || !bsrVal)) ||
      (nnzb32 > 0 && (!bsrColInd32 || !bsrVal32)))
    return SPMM_STATUS_INVALID_VALUE;
  spmm_context* ctx = handle;
  const int R = 32 / blockDim, shift = __builtin_ctz(R);
  const int mb32 = (mb + R - 1) / R;
  if (hipMemsetAsync(bsrVal32, 0, (size_t)nnzb32 * 1024 * sizeof(float), ctx->stream) != hipSuccess)
    return SPMM_STATUS_EXECUTION_FAILED;
  if (nnzb == 0 || mb32 == 0) return SPMM_STATUS_SUCCESS;
  const size_t need = 32 + (size_t)nnzb * 8;
  if (spmm_status_t st = spmm::ensure_workspace(ctx, need); st != SPMM_STATUS_SUCCESS) return st;
  char* ws = static_cast<char*>(ctx->ws);
  int* bad = reinterpret_cast<int*>(ws);
  int* map_k = reinterpret_cast<int*>(ws + 32);
  int* map_off = map_k + nnzb;
  hipLaunchKernelGGL(reblock32_kernel<true>, dim3((mb32 + 3) / 4), dim3(kWG), 0, ctx->stream, mb,
                     R, shift, bsrRowPtr, bsrColInd, nullptr, bsrRowPtr32, bsrColInd32, map_k,
                     map_off, blockDim, dir == SPMM_DIRECTION_ROW ? 1 : 0, bad);
  const long long total = (long long)nnzb * blockDim * blockDim;
  const long long blocks = std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(reblock32_values_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                     total, blockDim, blockDim * blockDim, bsrVal, map_k, map_off, bsrVal32);
  return spmm::from_hip(hipGetLastError());
}

}  // extern "C"
