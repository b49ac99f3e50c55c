// f64_kernels.hip — double-precision forms of both paths.
//
// The reference's operator templates take any T (gespmm_csrmm<T>,
// gespmm_csrmm.h:422; rocsparse_bsrmm_template<T>, rocsparse_bsrmm.h:102-108,
// whose impl carries a double myfma overload, rocsparse_bsrmm_impl.h:10);
// its drivers instantiate float only. These kernels give T = double the same
// semantics (C = alpha*A*B + beta*C, any storage order, index base 0/1) on
// the VALU in fp64: correctness-first, not tuned.
//  * CSR: one wave per row and 64-column tile, a sequential FMA chain in CSR
//    order per output element (the reference's accumulation order).
//  * BSR: one thread per output element of a block row, blocks in order and
//    k = 0..bs-1 inside each.
#include <hip/hip_runtime.h>

#include "context.hpp"

namespace {

__device__ __forceinline__ double epi64(double acc, double alpha, double beta, const double* p) {
  return beta == 0.0 ? alpha * acc : __builtin_fma(beta, *p, alpha * acc);
}

__global__ __launch_bounds__(256) void csr_f64_kernel(int m, int n, const int* __restrict__ rowptr,
                                                      const int* __restrict__ colind,
                                                      const double* __restrict__ val, int base,
                                                      const double* __restrict__ B, int ldb,
                                                      bool brow, double alpha, double beta,
                                                      double* __restrict__ C, int ldc, bool crow) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int j = blockIdx.y * 64 + lane;
  if (row >= m || j >= n) return;
  const int s = rowptr[row] - base, e = rowptr[row + 1] - base;
  double acc = 0.0;
  for (int p = s; p < e; ++p) {
    const size_t c = (size_t)(colind[p] - base);
    acc = __builtin_fma(val[p], brow ? B[c * ldb + j] : B[(size_t)j * ldb + c], acc);
  }
  double* out = crow ? C + (size_t)row * ldc + j : C + (size_t)j * ldc + row;
  *out = epi64(acc, alpha, beta, out);
}

__global__ __launch_bounds__(256) void bsr_f64_kernel(int mb, int n, int bs, bool rowdir,
                                                      const int* __restrict__ rowptr,
                                                      const int* __restrict__ colind,
                                                      const double* __restrict__ val,
                                                      const double* __restrict__ B, int ldb,
                                                      bool brow, double alpha, double beta,
                                                      double* __restrict__ C, int ldc, bool crow) {
  const int jj = threadIdx.x & 63;
  const int rl = threadIdx.x >> 6;
  const int br = blockIdx.x;
  const int j = blockIdx.y * 64 + jj;
  if (j >= n) return;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const size_t bs2 = (size_t)bs * bs;
  for (int rr = rl; rr < bs; rr += 4) {
    double acc = 0.0;
    for (int k = k0; k < k1; ++k) {
      const size_t bc = (size_t)colind[k] * bs;
      const double* ab = val + (size_t)k * bs2;
      for (int c = 0; c < bs; ++c) {
        const double av = rowdir ? ab[rr * bs + c] : ab[c * bs + rr];
        const double bv = brow ? B[(bc + c) * ldb + j] : B[(size_t)j * ldb + bc + c];
        acc = __builtin_fma(av, bv, acc);
      }
    }
    const size_t row = (size_t)br * bs + rr;
    double* p = crow ? C + row * ldc + j : C + (size_t)j * ldc + row;
    *p = epi64(acc, alpha, beta, p);
  }
}

}  // namespace

namespace spmm {

spmm_status_t launch_csrmm_f64(spmm_context* ctx, int m, int n, const int* rowptr,
                               const int* colind, const double* val, int base, const double* B,
                               int ldb, bool brow, double alpha, double beta, double* C, int ldc,
                               bool crow) {
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const int slot = timing_begin(ctx);
  hipLaunchKernelGGL(csr_f64_kernel, dim3((m + 3) / 4, (n + 63) / 64), dim3(256), 0, ctx->stream,
                     m, n, rowptr, colind, val, base, B, ldb, brow, alpha, beta, C, ldc, crow);
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsrmm_f64(spmm_context* ctx, spmm_direction_t dir, int mb, int n, int bs,
                               const int* rowptr, const int* colind, const double* val,
                               const double* B, int ldb, bool brow, double alpha, double beta,
                               double* C, int ldc, bool crow) {
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const int slot = timing_begin(ctx);
  hipLaunchKernelGGL(bsr_f64_kernel, dim3(mb, (n + 63) / 64), dim3(256), 0, ctx->stream, mb, n, bs,
                     dir == SPMM_DIRECTION_ROW, rowptr, colind, val, B, ldb, brow, alpha, beta, C,
                     ldc, crow);
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

}  // namespace spmm
