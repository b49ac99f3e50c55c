// group_kernels.hip — the device merge of the group analyses (spmm_bsr16_group_analysis_f16
// / spmm_bsr32_group_analysis_f32, group.cpp; DESIGN.md §4, "The grouped stream").
//
// A group is W adjacent block rows. Its entries are the union of the rows' nonzero block
// columns, each block column J expanded to the columns c its holders' column masks mark,
// in (J, c) order, cut into items of E entries (16 at bs 16, 8 at bs 32; the last item
// padded with row -1). One wave merges one group:
//  * a window holds the next L = 64 / W block columns of each row (lane w * L + i: row w,
//    element i);
//  * the cut is the least last element over the rows that continue past their window;
//    every element <= cut is accepted (no row holds a smaller one beyond its window), at
//    least a whole window of one row per step;
//  * each accepted element finds J in the other rows' windows (binary searches in LDS);
//    the first row holding J (the "first holder") owns union step J and ranks it by
//    ballot: its rank is the number of first holders below J, summed over the rows;
//  * union step r gets popcount(OR of the holders' masks) entries; a wave scan places
//    them after the entries so far, and (PASS 2) the lanes write 64 entries at a time:
//    the B row J * BS + c and, per row w of the group, the block holding (J, c) (-1:
//    none, or that block's column c is zero).
// PASS 1 counts the items, records the largest block column and flags a bad group with
// INT_MIN: a row pointer out of order (rp[0] != 0, decreasing, past nnzb, rp[mb] !=
// nnzb), a negative or oversized block column, or block columns not strictly increasing
// within a row (the contract: sorted per block row, no duplicates). Round 4's form was
// one thread per group walking the rows serially (1.45 ms for PASS 2 on the reddit
// stand-in at bs 32, 3,641 groups: 14 workgroups for 256 CUs).
#include <hip/hip_runtime.h>

#include <climits>

#include "context.hpp"

namespace {

__device__ __forceinline__ int wave_incl_scan(int x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Position of the k-th (from 0) set bit of m; m has more than k bits set.
__device__ __forceinline__ int nth_set_bit(unsigned m, int k) {
  int pos = 0;
#pragma unroll
  for (int s = 16; s > 0; s >>= 1) {
    const unsigned lo = m & ((1u << s) - 1u);
    const int c = __builtin_popcount(lo);
    if (k >= c) {
      k -= c;
      m >>= s;
      pos += s;
    } else {
      m = lo;
    }
  }
  return pos;
}

template <int W, int BS, bool PASS2>
__global__ __launch_bounds__(64) void grp_build_kernel(int mb, int nnzb, int ngroups,
                                                       const int* __restrict__ rp,
                                                       const int* __restrict__ ci,
                                                       const unsigned* __restrict__ mk,
                                                       int* __restrict__ cnt, int* __restrict__ maxj,
                                                       const int* __restrict__ item_ptr,
                                                       int* __restrict__ rows, int* __restrict__ src) {
  constexpr int L = 64 / W;  // window elements per row
  constexpr unsigned kAll = BS == 32 ? 0xffffffffu : 0xffffu;
  constexpr int E = BS == 16 ? 16 : 8;
  constexpr int kMaxJ = INT_MAX / BS;  // J * BS + c stays an int
  constexpr unsigned long long kRow = (1ull << L) - 1ull;
  __shared__ int sJ[64];          // window: block column (INT_MAX past the row's end)
  __shared__ unsigned sM[64];     // window: column mask of an accepted element
  __shared__ int sK[64];          // window: block index
  __shared__ int sU[64];          // union step r: block column
  __shared__ unsigned sUm[64];    // union step r: OR of the holders' masks
  __shared__ int sP[64];          // union step r: first entry (exclusive scan)
  __shared__ signed char sH[64][W];  // union step r: window lane of row w holding it, or -1
  const int g = blockIdx.x;
  const int lane = threadIdx.x;
  const int w = lane / L, i = lane % L;
  // the row pointer is checked before it indexes the block columns
  int rb = 0, re = 0;
  bool bad = false;
  if (lane < W) {
    const int br = g * W + lane;
    if (br < mb) {
      rb = rp[br];
      re = rp[br + 1];
    }
    bad = re < rb || rb < 0 || re > nnzb;
    if (lane == 0) bad |= (g == 0 && rp[0] != 0) || (g == ngroups - 1 && rp[mb] != nnzb);
  }
  bool fail = __builtin_amdgcn_ballot_w64(bad) != 0ull;
  int rc = __shfl(rb, w, 64), rend = __shfl(re, w, 64);  // this lane's row: cursor, end
  if (fail) rc = rend = 0;
  long long e = 0;  // entries so far
  int hi = -1;
  int lastJ = -1;   // the row's last accepted block column
  const long long base = PASS2 ? (long long)item_ptr[g] * E : 0;
  const long long lim = PASS2 ? (long long)item_ptr[g + 1] * E : 0;
  for (;;) {
    const int idx = rc + i;
    const bool valid = idx < rend;
    const int J = valid ? ci[idx] : INT_MAX;
    const int prev = __shfl_up(J, 1, 64);
    const bool wrong = valid && (J < 0 || J >= kMaxJ || J <= (i == 0 ? lastJ : prev));
    if (__builtin_amdgcn_ballot_w64(wrong)) {
      fail = true;
      break;
    }
    const bool more = rc + L < rend;
    int cut = INT_MAX;
#pragma unroll
    for (int r = 0; r < W; ++r) {
      const int x = __builtin_amdgcn_readlane(more && i == L - 1 ? J : INT_MAX, r * L + L - 1);
      cut = min(cut, x);
    }
    const bool acc = valid && J <= cut;
    const unsigned long long accm = __builtin_amdgcn_ballot_w64(acc);
    if (accm == 0ull) break;  // every row consumed
    sJ[lane] = J;
    sM[lane] = acc ? (mk[idx] & kAll) : 0u;
    sK[lane] = idx;
    __syncthreads();
    // holders of J in every row's window (own row: this lane)
    int pos[W];
    bool fnd[W];
    bool first = acc;
#pragma unroll
    for (int r = 0; r < W; ++r) {
      int lo = 0;
#pragma unroll
      for (int s = L / 2; s > 0; s >>= 1)
        if (sJ[r * L + lo + s - 1] < J) lo += s;
      if (sJ[r * L + lo] < J) ++lo;  // lo in [0, L]: the elements of row r below J
      pos[r] = lo;
      fnd[r] = lo < L && sJ[r * L + lo] == J;
      if (fnd[r] && r < w) first = false;
    }
    const unsigned long long fm = __builtin_amdgcn_ballot_w64(first);
    int rank = 0;
#pragma unroll
    for (int r = 0; r < W; ++r)
      rank += __builtin_popcountll(fm & (((1ull << pos[r]) - 1ull) << (r * L)));
    if (first) {
      unsigned um = 0u;
#pragma unroll
      for (int r = 0; r < W; ++r) {
        if (fnd[r]) um |= sM[r * L + pos[r]];
        sH[rank][r] = fnd[r] ? (signed char)(r * L + pos[r]) : (signed char)-1;
      }
      sU[rank] = J;
      sUm[rank] = um;
    }
    __syncthreads();
    const int U = __builtin_popcountll(fm);
    const int n = lane < U ? __builtin_popcount(sUm[lane]) : 0;
    const int incl = wave_incl_scan(n, lane);
    const int T = __builtin_amdgcn_readlane(incl, 63);
    hi = max(hi, sU[U - 1]);
    if constexpr (PASS2) {
      sP[lane] = incl - n;
      __syncthreads();
      for (int t0 = 0; t0 < T; t0 += 64) {
        const int t = t0 + lane;
        const long long x = base + e + t;
        if (t < T && x < lim) {
          int r = 0;  // the last union step starting at or before t
#pragma unroll
          for (int s = 32; s > 0; s >>= 1)
            if (r + s < U && sP[r + s] <= t) r += s;
          const int c = nth_set_bit(sUm[r], t - sP[r]);
          rows[x] = sU[r] * BS + c;
#pragma unroll
          for (int q = 0; q < W; ++q) {
            const int h = sH[r][q];
            src[x * W + q] = h >= 0 && ((sM[h] >> c) & 1u) ? sK[h] : -1;
          }
        }
      }
    }
    e += T;
    // advance every row past its accepted elements
    const int took = __builtin_popcountll(accm & (kRow << (w * L)));
    const int lastacc = __shfl(J, w * L + (took > 0 ? took - 1 : 0), 64);
    if (took > 0) lastJ = lastacc;
    rc += took;
    __syncthreads();  // the next window overwrites the LDS
  }
  if constexpr (PASS2) {
    // pad the last item with row -1, no source
    const long long pad = (E - e % E) % E;
    if (lane < pad) {
      const long long x = base + e + lane;
      if (x < lim) {
        rows[x] = -1;
#pragma unroll
        for (int q = 0; q < W; ++q) src[x * W + q] = -1;
      }
    }
  } else {
    if (lane == 0) {
      const long long items = (e + E - 1) / E;
      cnt[g] = fail ? 0 : (items > INT_MAX ? INT_MAX : (int)items);
      maxj[g] = fail ? INT_MIN : hi;
    }
  }
}

// wmask[item][w], bit e: entry e of the item has a source block in row w (the
// MFMAs wave w runs at bs 32, the B values its fragments keep at bs 16).
template <int E>
__global__ __launch_bounds__(256) void grp_wmask_kernel(long long nwork, int W,
                                                        const int* __restrict__ src,
                                                        unsigned* __restrict__ wmask) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= nwork) return;
  const long long item = t / W;
  const int w = (int)(t - item * W);
  unsigned m = 0u;
#pragma unroll
  for (int e = 0; e < E; ++e) m |= (src[(item * E + e) * W + w] >= 0 ? 1u : 0u) << e;
  wmask[t] = m;
}

// One workgroup: stats[0] = max maxj (-1 when n = 0), stats[1] = any INT_MIN.
__global__ __launch_bounds__(1024) void grp_stats_kernel(const int* __restrict__ maxj, int n,
                                                         int* __restrict__ stats) {
  __shared__ int smax[16], sbad[16];
  int hi = -1, bad = 0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const int x = maxj[i];
    bad |= x == INT_MIN;
    hi = max(hi, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    hi = max(hi, __shfl_xor(hi, o));
    bad |= __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    smax[threadIdx.x >> 6] = hi;
    sbad[threadIdx.x >> 6] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) {
      hi = max(hi, smax[w]);
      bad |= sbad[w];
    }
    stats[0] = hi;
    stats[1] = bad;
  }
}

}  // namespace

namespace spmm {

spmm_status_t launch_grp_build(spmm_context* ctx, int W, int BS, bool pass2, int mb, int nnzb,
                               int ngroups, const int* rp, const int* ci, const unsigned* mk,
                               int* cnt, int* maxj, const int* item_ptr, int* rows, int* src) {
  if (ngroups == 0) return SPMM_STATUS_SUCCESS;
  const dim3 grid(ngroups);
#define GRP_BUILD(W_, BS_)                                                                     \
  do {                                                                                         \
    if (pass2)                                                                                 \
      hipLaunchKernelGGL((grp_build_kernel<W_, BS_, true>), grid, dim3(64), 0, ctx->stream, mb, \
                         nnzb, ngroups, rp, ci, mk, cnt, maxj, item_ptr, rows, src);            \
    else                                                                                       \
      hipLaunchKernelGGL((grp_build_kernel<W_, BS_, false>), grid, dim3(64), 0, ctx->stream,   \
                         mb, nnzb, ngroups, rp, ci, mk, cnt, maxj, item_ptr, rows, src);        \
  } while (0)
  if (BS == 16) {
    if (W == 8) GRP_BUILD(8, 16);
    else if (W == 4) GRP_BUILD(4, 16);
    else GRP_BUILD(2, 16);
  } else {
    if (W == 4) GRP_BUILD(4, 32);
    else GRP_BUILD(2, 32);
  }
#undef GRP_BUILD
  return from_hip(hipGetLastError());
}

spmm_status_t launch_grp_wmask(spmm_context* ctx, long long nitems, int W, int E, const int* src,
                               unsigned* wmask) {
  const long long nwork = nitems * W;
  if (nwork == 0) return SPMM_STATUS_SUCCESS;
  const dim3 grid((unsigned)((nwork + 255) / 256));
  if (E == 16)
    hipLaunchKernelGGL(grp_wmask_kernel<16>, grid, dim3(256), 0, ctx->stream, nwork, W, src, wmask);
  else
    hipLaunchKernelGGL(grp_wmask_kernel<8>, grid, dim3(256), 0, ctx->stream, nwork, W, src, wmask);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_grp_stats(spmm_context* ctx, const int* maxj, int n, int* stats) {
  hipLaunchKernelGGL(grp_stats_kernel, dim3(1), dim3(1024), 0, ctx->stream, maxj, n, stats);
  return from_hip(hipGetLastError());
}

}  // namespace spmm
