// group_kernels.hip — the device merge and the bs 32 A-fragment fill of the group analyses
// (spmm_bsr16_group_analysis_f16 / spmm_bsr32_group_analysis_f32, group.cpp; DESIGN.md §4,
// "The grouped stream").
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
#include <cstdint>

#include "context.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// A fragments of the grouped bs 32 stream (layout per (item, wave w): [32 rows][8 entries]
// fp32, A[row][entry] of block row w of the group; zero where src = -1). One wave per run of
// kFill32Items consecutive items of one w: its 64 entries (lane t: item t / 8, entry t % 8)
// name the blocks holding them; each distinct block is read once, whole and coalesced (lane
// (j, h): row j, columns 16h .. 16h + 15 of a ROW block; column j, rows 16h .. of a COLUMN
// block; the next block's loads in flight while this one is placed), transposed into LDS
// (column c at c * 33, conflict-free) and its entries' columns copied into the run's
// fragments in LDS, which go out as 1-KB coalesced stores. Round 4's form gathered each
// entry's column straight from the block (32 lines of 128 B for 128 B used); both run
// 1.8 ms on the reddit stand-in (3.0 on products): every held block's 4 KB are read once
// either way and the fragments written, about 9 GB at 5 TB/s (16.6 GB at 5.4 on
// products), so the gain is in L2 requests, not time. At bs 16 (below) the chunked form
// took the fill from 1.26 to 0.86 ms on products.
#ifndef SPMM_FILL32_ITEMS
#define SPMM_FILL32_ITEMS 8
#endif
#ifndef SPMM_FILL32_RING
#define SPMM_FILL32_RING 3
#endif
// items per wave (at most 8: 64 entries) and blocks in flight per wave; 4 items or 4 blocks
// ran the same times (profiles/r05c/ab_fill32/): the fill is bound by its HBM traffic
constexpr int kFill32Items = SPMM_FILL32_ITEMS;
constexpr int kFill32Ring = SPMM_FILL32_RING;

__global__ __launch_bounds__(64) void bsr32_grp_fill_kernel(long long nitems, int W, int rowdir,
                                                            const int* __restrict__ rows,
                                                            const int* __restrict__ src,
                                                            const float* __restrict__ val,
                                                            float* __restrict__ afrag) {
  __shared__ float blk[32 * 33];                      // [column][row], padded
  __shared__ f32x4 frag[kFill32Items * 256 / 4];      // [item][row][entry]
  const int lane = threadIdx.x;
  const long long u = blockIdx.x;
  const int w = (int)(u % W);
  const long long item0 = (u / W) * kFill32Items;
  const int nf = (int)min((long long)kFill32Items, nitems - item0);
  const long long it = item0 + (lane >> 3);
  const bool mine = (lane >> 3) < kFill32Items;
  const int row = mine && it < nitems ? rows[it * 8 + (lane & 7)] : -1;
  const int k = row >= 0 ? src[(it * 8 + (lane & 7)) * W + w] : -1;
  const int c = row & 31;
#pragma unroll
  for (int q = 0; q < kFill32Items; ++q) frag[q * 64 + lane] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int j = lane >> 1, h = lane & 1;
  const size_t off = (size_t)j * 32 + 16 * h;  // 16 floats: row (ROW) or column (COLUMN) j
  // their LDS places: ROW A[j][16h + i] -> column 16h + i; COLUMN A[16h + i][j] -> column j
  const int pbase = rowdir ? 16 * h * 33 + j : j * 33 + 16 * h, pstep = rowdir ? 33 : 1;
  // a ring of kFill32Ring blocks in flight: slot s is placed, then refilled with the next
  // block not yet issued (static slot indices: no register moves wait on a load)
  f32x4 ring[kFill32Ring][4];
  int rb[kFill32Ring];
  unsigned long long unissued = __builtin_amdgcn_ballot_w64(k >= 0);
  // every slot loads unconditionally (one resource per block; none left: an offset past
  // its end, zeros without a memory access), so hipcc counts the waits inside the ring
  // (vmcnt(8) for the slot placed while two are in flight; only the loop head waits more)
  auto issue = [&](int s) {
    rb[s] = unissued ? __builtin_amdgcn_readlane(k, __builtin_ctzll(unissued)) : -1;
    unissued &= ~__builtin_amdgcn_ballot_w64(k == rb[s]);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(val + (size_t)max(rb[s], 0) * 1024), 0, 4096, 0x00020000);
    const unsigned o = rb[s] >= 0 ? (unsigned)off * 4u : 0x80000000u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      ring[s][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16u * q, 0, 0));
  };
  auto place = [&](const f32x4 (&x)[4], int b) {
    __syncthreads();  // the previous block's columns are read
#pragma unroll
    for (int i = 0; i < 16; ++i) blk[pbase + i * pstep] = x[i >> 2][i & 3];
    __syncthreads();
    // the block's entries, two per step: lanes 0-31 the first, 32-63 the second
    unsigned long long todo = __builtin_amdgcn_ballot_w64(k == b);
    while (todo) {
      const int ta = __builtin_ctzll(todo);
      todo &= todo - 1ull;
      const int tb = todo ? __builtin_ctzll(todo) : -1;
      if (tb >= 0) todo &= todo - 1ull;
      const int t = lane < 32 ? ta : tb;
      const int ct = __builtin_amdgcn_readlane(c, ta);
      const int cb = tb >= 0 ? __builtin_amdgcn_readlane(c, tb) : 0;
      if (t >= 0) {
        const int r = lane & 31;
        const float v = blk[(lane < 32 ? ct : cb) * 33 + r];
        reinterpret_cast<float*>(frag)[(t >> 3) * 256 + r * 8 + (t & 7)] = v;
      }
    }
  };
#pragma unroll
  for (int s = 0; s < kFill32Ring; ++s) issue(s);
  bool more = rb[0] >= 0;
  while (more) {
#pragma unroll
    for (int s = 0; s < kFill32Ring; ++s) {
      if (rb[s] < 0) {
        more = false;
        break;
      }
      place(ring[s], rb[s]);
      issue(s);
    }
  }
  __syncthreads();
  f32x4* dst = reinterpret_cast<f32x4*>(afrag);
  for (int f = 0; f < nf; ++f)
    dst[((item0 + f) * W + w) * 64 + lane] = frag[f * 64 + lane];
}

// Round 6: the analysis in one pass over A. The column masks (grp_mask32_kernel, in the size
// query) also write, for ROW blocks, a compact column-major copy of each block's nonzero
// columns: block k's column c, when nonzero, at cols[k * 1024 + 32 p ..], p the rank of c
// among the block's nonzero columns (a transient slot of 4 KB per block, of which only the
// nonzero columns are written). The fill (bsr32_grp_fillc_kernel) then reads 128 B per entry
// from it (COLUMN blocks: straight from the values, whose columns are contiguous) instead of
// every held block's 4 KB: the analysis read A twice, once for the masks and once in the fill
// above (1.24 + 1.80 ms of 3.36 on the reddit stand-in, 2.01 + 3.08 of 5.45 on products,
// profiles/r05c/grp_b6_mask32_tried.txt). The fragments are the same bytes either way.
// One wave per block, four per workgroup; ROW: lane (j, h) loads row j, columns 16h .. 16h + 15
// (four 16-B loads), a ballot per column pair (i, 16 + i) gives both bits, and each nonzero
// column goes out as one 128-B line per half-wave. COLUMN: lane L loads floats 16L .. 16L + 15
// = column L / 2, half L & 1; one ballot.
__global__ __launch_bounds__(256) void grp_mask32_kernel(long long nnzb, int rowdir,
                                                         const float* __restrict__ val,
                                                         unsigned* __restrict__ masks,
                                                         float* __restrict__ cols) {
  const int lane = threadIdx.x & 63;
  const long long k = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= nnzb) return;
  const float* blk = val + (size_t)k * 1024;
  unsigned msk = 0;
  if (rowdir) {
    const int j = lane & 31, h = lane >> 5;
    f32x4 x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = *reinterpret_cast<const f32x4*>(blk + j * 32 + 16 * h + 4 * q);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned long long b =
          __builtin_amdgcn_ballot_w64((__float_as_uint(x[i >> 2][i & 3]) & 0x7fffffffu) != 0u);
      msk |= ((unsigned)b != 0u ? 1u : 0u) << i;
      msk |= ((unsigned)(b >> 32) != 0u ? 1u : 0u) << (16 + i);
    }
    if (cols) {
      float* dst = cols + (size_t)k * 1024 + j;
      const unsigned below = msk & ((1u << (16 * h)) - 1u);  // columns of the other half first
      int p = __builtin_popcount(below);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if ((msk >> (16 * h + i)) & 1u) {  // uniform over the half-wave
          dst[32 * p] = x[i >> 2][i & 3];
          ++p;
        }
      }
    }
  } else {
    f32x4 x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = *reinterpret_cast<const f32x4*>(blk + 16 * lane + 4 * q);
    unsigned t = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) t |= __float_as_uint(x[q][e]) & 0x7fffffffu;
    const unsigned long long b = __builtin_amdgcn_ballot_w64(t != 0u);
#pragma unroll
    for (int c = 0; c < 32; ++c) msk |= (((b >> (2 * c)) & 3ull) != 0ull ? 1u : 0u) << c;
  }
  if (lane == 0) masks[k] = msk;
}

// The fill from columns: one wave per run of kFill32Items items of one w, lane t naming entry
// t (item t / 8, entry t % 8) and the place of its column (masks: the compact copy's rank;
// none: a COLUMN block's own column). Eight lanes read one entry's 128 B (lane q: rows
// 4q .. 4q + 3), eight entries per load instruction, all of the run's loads in flight
// together; the run's fragments are assembled in LDS and go out as 1-KB coalesced stores.
__global__ __launch_bounds__(64) void bsr32_grp_fillc_kernel(long long nitems, int W,
                                                             const int* __restrict__ rows,
                                                             const int* __restrict__ src,
                                                             const float* __restrict__ cols,
                                                             const unsigned* __restrict__ masks,
                                                             float* __restrict__ afrag) {
  __shared__ f32x4 frag[kFill32Items * 256 / 4];  // [item][row][entry]
  const int lane = threadIdx.x;
  const long long u = blockIdx.x;
  const int w = (int)(u % W);
  const long long item0 = (u / W) * kFill32Items;
  const int nf = (int)min((long long)kFill32Items, nitems - item0);
  const long long it = item0 + (lane >> 3);
  const bool mine = (lane >> 3) < kFill32Items;
  const int row = mine && it < nitems ? rows[it * 8 + (lane & 7)] : -1;
  const int k = row >= 0 ? src[(it * 8 + (lane & 7)) * W + w] : -1;
  const int c = row & 31;
  // the entry's column: cols + 1024 k + 32 rank (k < 2^31: the offset fits 64 bits as lo / hi)
  const int rank = k >= 0 ? (masks ? __builtin_popcount(masks[k] & ((1u << c) - 1u)) : c) : 0;
#pragma unroll
  for (int q = 0; q < kFill32Items; ++q) frag[q * 64 + lane] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q = lane & 7, er = lane >> 3;
  int kt[kFill32Items];
  f32x4 x[kFill32Items];
#pragma unroll
  for (int r = 0; r < kFill32Items; ++r) {
    const int t = r * 8 + er;  // item r of the run, entry er
    kt[r] = __shfl(k, t, 64);
    const int rk = __shfl(rank, t, 64);
    x[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kt[r] >= 0)
      x[r] = *reinterpret_cast<const f32x4*>(cols + (size_t)kt[r] * 1024 + 32 * rk + 4 * q);
  }
  __syncthreads();  // the zeroed fragments
  float* fr = reinterpret_cast<float*>(frag);
#pragma unroll
  for (int r = 0; r < kFill32Items; ++r)
    if (kt[r] >= 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) fr[r * 256 + (4 * q + i) * 8 + er] = x[r][i];
  __syncthreads();
  f32x4* dst = reinterpret_cast<f32x4*>(afrag);
  for (int f = 0; f < nf; ++f)
    dst[((item0 + f) * W + w) * 64 + lane] = frag[f * 64 + lane];
}

// A fragments of the grouped bs 16 fp16 stream (layout per (item, wave w): 128 uint32, lane
// l of the product's wave holding A[l & 15][4 (l >> 4) .. + 3] as fp16 x 4, i.e. half
// 64 (e >> 2) + 4 r + (e & 3) for row r, entry e). One wave per run of kFill16Items items of
// one w, lane t owning entry t (item t / 16, entry t % 16). The run's distinct blocks are read
// kFill16Chunk at a time, whole and coalesced (lane (j, q): 4 halves of row j (ROW) or column
// j (COLUMN) at 4q), all in flight together, and transposed into LDS (column c at c * 17
// halves); then every lane copies the 16 rows of its entry's column, if its block is in the
// chunk, into the run's fragments in LDS, which are stored 512 B at a time. Two barriers
// per chunk of blocks: a form that placed one block at a time (two barriers and a ballot
// walk per block) ran 1.12 ms on the products stand-in, round 4's column gathers 1.26 ms.
constexpr int kFill16Items = 4;
constexpr int kFill16Chunk = 8;

__global__ __launch_bounds__(64) void bsr16_grp_fill_kernel(long long nitems, int W, int rowdir,
                                                            const int* __restrict__ rows,
                                                            const int* __restrict__ src,
                                                            const uint16_t* __restrict__ val,
                                                            unsigned* __restrict__ afrag) {
  __shared__ uint16_t blk[kFill16Chunk][16 * 17];      // per block: [column][row], padded
  __shared__ uint2 frag[kFill16Items * 64];            // [item][lane of the product's wave]
  const int lane = threadIdx.x;
  const long long u = blockIdx.x;
  const int w = (int)(u % W);
  const long long item0 = (u / W) * kFill16Items;
  const int nf = (int)min((long long)kFill16Items, nitems - item0);
  const long long it = item0 + (lane >> 4);
  const int row = it < nitems ? rows[it * 16 + (lane & 15)] : -1;
  const int k = row >= 0 ? src[(it * 16 + (lane & 15)) * W + w] : -1;
  const int c = row & 15;
#pragma unroll
  for (int q = 0; q < kFill16Items; ++q) frag[q * 64 + lane] = uint2{0u, 0u};
  const int j = lane >> 2, q4 = lane & 3;
  const unsigned off = 2u * (unsigned)(j * 16 + 4 * q4);  // 4 halves: row (ROW) or column (COLUMN) j
  // ROW A[j][4q + i] -> column 4q + i; COLUMN A[4q + i][j] -> column j
  const int pbase = rowdir ? 4 * q4 * 17 + j : j * 17 + 4 * q4, pstep = rowdir ? 17 : 1;
  // this lane's entry: its 16 halves' places in the run's fragments
  const int e = lane & 15;
  const int fbase = (lane >> 4) * 256 + 64 * (e >> 2) + (e & 3);
  unsigned long long unissued = __builtin_amdgcn_ballot_w64(k >= 0);
  while (unissued) {
    int bk[kFill16Chunk];
    uint2 x[kFill16Chunk];
#pragma unroll
    for (int d = 0; d < kFill16Chunk; ++d) {
      // every slot loads (none left: an offset past the resource's end, zeros without a
      // memory access)
      bk[d] = unissued ? __builtin_amdgcn_readlane(k, __builtin_ctzll(unissued)) : -1;
      unissued &= ~__builtin_amdgcn_ballot_w64(k == bk[d]);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(val + (size_t)max(bk[d], 0) * 256), 0, 512, 0x00020000);
      x[d] = __builtin_bit_cast(
          uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, bk[d] >= 0 ? off : 0x80000000u, 0, 0));
    }
    __syncthreads();  // the previous chunk's columns are read
#pragma unroll
    for (int d = 0; d < kFill16Chunk; ++d)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        blk[d][pbase + i * pstep] = (uint16_t)((i < 2 ? x[d].x : x[d].y) >> (16 * (i & 1)));
    __syncthreads();
    int slot = -1;
#pragma unroll
    for (int d = 0; d < kFill16Chunk; ++d)
      if (bk[d] >= 0 && k == bk[d]) slot = d;
    if (slot >= 0) {
      const uint16_t* col = &blk[slot][c * 17];
      uint16_t* dst = reinterpret_cast<uint16_t*>(frag) + fbase;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[4 * r] = col[r];
    }
  }
  __syncthreads();
  uint2* dst = reinterpret_cast<uint2*>(afrag);
  for (int f = 0; f < nf; ++f) dst[((item0 + f) * W + w) * 64 + lane] = frag[f * 64 + lane];
}

// Column masks of bs 16 fp16 blocks for the group analysis (masks only; spmm_bsr16_analysis_f16
// keeps bsr16_analysis_kernel, which also writes the column-major copy): bit c set when column
// c holds a value other than +-0 (NaN and inf included). A half-wave per block, one 16-B load
// per lane (8 halves: ROW row l / 2, columns 8 (l & 1) ..; COLUMN column l / 2, rows 8 (l & 1)
// ..), kMask16Pairs block pairs per wave in flight. ROW: the 16 lanes of each parity OR their
// flags (4 xor shuffles); COLUMN: one ballot. 16-B aligned values only (else the older kernel).
constexpr int kMask16Pairs = 8;

__global__ __launch_bounds__(256) void grp_mask16_kernel(long long nnzb, int rowdir,
                                                         const uint16_t* __restrict__ val,
                                                         unsigned* __restrict__ masks) {
  const int lane = threadIdx.x & 63;
  const long long k0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * (2 * kMask16Pairs);
  if (k0 >= nnzb) return;
  const int half = lane >> 5, l = lane & 31;
  uint4 xs[kMask16Pairs];
#pragma unroll
  for (int p = 0; p < kMask16Pairs; ++p) {
    const long long k = min(k0 + 2 * p + half, nnzb - 1);  // past the end: loaded, not stored
    xs[p] = *reinterpret_cast<const uint4*>(val + (size_t)k * 256 + 8 * l);
  }
#pragma unroll
  for (int p = 0; p < kMask16Pairs; ++p) {
    const long long k = k0 + 2 * p + half;
    const unsigned w[4] = {xs[p].x, xs[p].y, xs[p].z, xs[p].w};
    unsigned f = 0u;  // bit i: half i of this lane's 8 is nonzero
#pragma unroll
    for (int i = 0; i < 4; ++i)
      f |= ((w[i] & 0x7fffu) != 0u ? 1u : 0u) << (2 * i) |
           ((w[i] & 0x7fff0000u) != 0u ? 1u : 0u) << (2 * i + 1);
    unsigned msk;
    if (rowdir) {
      unsigned o = f;
#pragma unroll
      for (int d = 2; d < 32; d <<= 1) o |= __shfl_xor(o, d, 64);
      msk = __shfl(o, 32 * half, 64) | (__shfl(o, 32 * half + 1, 64) << 8);
    } else {
      const unsigned bb = (unsigned)(__builtin_amdgcn_ballot_w64(f != 0u) >> (32 * half));
      msk = 0u;
#pragma unroll
      for (int c = 0; c < 16; ++c) msk |= ((bb >> (2 * c)) & 3u ? 1u : 0u) << c;
    }
    if (l == 0 && k < nnzb) masks[k] = msk;
  }
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

spmm_status_t launch_bsr16_grp_fill(spmm_context* ctx, long long nitems, int W, spmm_direction_t dir,
                                    const int* rows, const int* src, const uint16_t* val,
                                    unsigned* afrag) {
  if (nitems == 0) return SPMM_STATUS_SUCCESS;
  const long long units = (nitems + kFill16Items - 1) / kFill16Items * W;
  hipLaunchKernelGGL(bsr16_grp_fill_kernel, dim3((unsigned)units), dim3(64), 0, ctx->stream, nitems,
                     W, dir == SPMM_DIRECTION_ROW ? 1 : 0, rows, src, val, afrag);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsr32_grp_fill(spmm_context* ctx, long long nitems, int W, spmm_direction_t dir,
                                    const int* rows, const int* src, const float* val,
                                    float* afrag) {
  if (nitems == 0) return SPMM_STATUS_SUCCESS;
  const long long units = (nitems + kFill32Items - 1) / kFill32Items * W;
  hipLaunchKernelGGL(bsr32_grp_fill_kernel, dim3((unsigned)units), dim3(64), 0, ctx->stream, nitems,
                     W, dir == SPMM_DIRECTION_ROW ? 1 : 0, rows, src, val, afrag);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_grp_mask32(spmm_context* ctx, spmm_direction_t dir, int nnzb, const float* val,
                                unsigned* masks, float* cols) {
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  hipLaunchKernelGGL(grp_mask32_kernel, dim3((unsigned)(((long long)nnzb + 3) / 4)), dim3(256), 0,
                     ctx->stream, (long long)nnzb, dir == SPMM_DIRECTION_ROW ? 1 : 0, val, masks,
                     dir == SPMM_DIRECTION_ROW ? cols : nullptr);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsr32_grp_fillc(spmm_context* ctx, long long nitems, int W, const int* rows,
                                     const int* src, const float* cols, const unsigned* masks,
                                     float* afrag) {
  if (nitems == 0) return SPMM_STATUS_SUCCESS;
  const long long units = (nitems + kFill32Items - 1) / kFill32Items * W;
  hipLaunchKernelGGL(bsr32_grp_fillc_kernel, dim3((unsigned)units), dim3(64), 0, ctx->stream, nitems,
                     W, rows, src, cols, masks, afrag);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_grp_mask16(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                const uint16_t* val, unsigned* masks) {
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  const long long per_block = 4 * 2 * kMask16Pairs;  // 4 waves, kMask16Pairs block pairs each
  hipLaunchKernelGGL(grp_mask16_kernel, dim3((unsigned)((nnzb + per_block - 1) / per_block)),
                     dim3(256), 0, ctx->stream, (long long)nnzb, dir == SPMM_DIRECTION_ROW ? 1 : 0,
                     val, masks);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_grp_stats(spmm_context* ctx, const int* maxj, int n, int* stats) {
  hipLaunchKernelGGL(grp_stats_kernel, dim3(1), dim3(1024), 0, ctx->stream, maxj, n, stats);
  return from_hip(hipGetLastError());
}

}  // namespace spmm
