// bsr_kernels.hip — Path B: BSR x dense on gfx950 (MI355X).
//
// Semantic target is cusparseSbsrmm (run_bsrmm.cu:160-165, bsrmm.cu:141-144):
//   C = alpha * A_bsr * op(B) + beta * C
// with DIRECTION_ROW / COLUMN block storage. The reference's own transcription
// of rocSPARSE (rocsparse_bsrmm_impl.h:315-389) indexes column tiles with
// blockDim.y instead of blockIdx.y (:326) and writes nothing for bs 16/32 at
// K <= 256, so it is not used as an oracle. The
// epilogue follows its rocSPARSE convention (impl.h:381-388): beta == 0 gives
// C = alpha*sum without reading C, else C = fma(beta, C, alpha*sum).
//
// Kernels:
//  * bs = 32, fp32: every nonzero block is an MFMA A-tile of
//    v_mfma_f32_32x32x2_f32. A wave owns 32 rows (the block row) x 32 output
//    columns; a block contributes 16 MFMAs. The k index inside an MFMA pair
//    is permuted (step s, lane half h -> k = 16h + s) so each lane's A
//    fragment is 16 contiguous floats of one block row (4 x dwordx4) and,
//    for column-major B, its B fragment is 16 contiguous floats too.
//  * bs = 16, fp32: v_mfma_f32_16x16x4_f32, k = 4q + s, 4 column tiles per
//    wave sharing the A fragment (one dwordx4 per block).
//  * bs = 16, fp16 A/B: v_mfma_f32_16x16x32_f16 consumes TWO blocks of the
//    block row per instruction (k 0-15 from block b, 16-31 from block b+1).
//  * any other bs: a VALU kernel with the same semantics.
// Fragments of block b+1 are loaded while block b's MFMAs issue.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "context.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float epi(float acc, float alpha, float beta, const float* p) {
  return beta == 0.f ? alpha * acc : __builtin_fmaf(beta, *p, alpha * acc);
}

// Waits (once, before the block loop) for the loads that filled a fragment
// buffer. Without it the loop header merges the prologue's loads with the
// back edge, and hipcc's waitcnt pass puts a conservative counted wait on the
// first MFMA that then also covers the prefetches issued in the same
// iteration (measured: the prefetch hid nothing; hot-L2 and cold B panels ran
// at the same 41 % of the MFMA peak).
__device__ __forceinline__ void settle(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void settle(f16x8& x) { asm volatile("" : "+v"(x)); }
template <typename T, int N>
__device__ __forceinline__ void settle(T (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) settle(x[i]);
}

// Wave-uniform block-column cursor over bsr_col_ind[k0, k1): 64 entries held
// one per lane, read with v_readlane (no dependent scalar load per block) and
// refilled in place every 64 blocks. The refill waits right away (asm use),
// so the common path after the branch carries no conservative vmcnt(0).
struct ColCursor {
  const int* colind;
  int k1, lane, base, vec;
  __device__ __forceinline__ ColCursor(const int* ci, int k0, int k1_, int lane_)
      : colind(ci), k1(k1_), lane(lane_), base(k0) {
    refill();
  }
  __device__ __forceinline__ void refill() {
    vec = colind[min(base + lane, max(k1 - 1, 0))];
    asm volatile("" : "+v"(vec));
  }
  // k must be visited in non-decreasing order.
  __device__ __forceinline__ int get(int k) {
    if (k - base >= 64) {
      base += 64 * ((k - base) >> 6);
      refill();
    }
    return __builtin_amdgcn_readlane(vec, k - base);
  }
};

// ---------------------------------------------------------------------------
// bs = 32 fp32 MFMA. Block = 4 waves, each wave a 32-column slice.
// ---------------------------------------------------------------------------
// VAR (tuning variants; kBsr32Default is the shipped one):
//   VAR & 3  pipeline: 0 = prefetch block k+1 into a second register set,
//            1 = fixed-role double buffer, 2 = load-use (no prefetch; the
//            other resident waves hide the latency)
//   VAR & 4  XCD-aware block-row order (neighbouring block rows share an L2)
//   VAR >> 3 minimum waves per SIMD requested from the register allocator
//            (0 = no bound). Measured on the reddit stand-in:
//            this kernel is bound by B-panel traffic beyond L2, so resident
//            waves (memory-level parallelism) decide its speed.
template <bool ROWDIR, bool BROW, bool CROW, int VAR>
__global__ __launch_bounds__(256, (VAR >> 3) ? (VAR >> 3) : 1) void bsr32_f32_mfma_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  int br = blockIdx.x;
  if constexpr ((VAR & 4) != 0) {
    // Round-robin dispatch puts block b on XCD b % 8: give each XCD a
    // contiguous range of block rows instead (bijective for any mb).
    const int q = mb / 8, rem = mb % 8, x = br % 8, i = br / 8;
    br = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + i;
  }
  const int j0 = (blockIdx.y * (blockDim.x >> 6) + wv) * 32;
  if (j0 >= n) return;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int jcol = j0 + r;
  const bool jok = jcol < n;
  const int jld = jok ? jcol : j0;

  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;

  ColCursor cc(colind, k0, k1, lane);
  auto load_frags = [&](int k, float (&fa)[16], float (&fb)[16]) {
    const int bc = cc.get(k);
    const float* ab = val + (size_t)k * 1024;
    if constexpr (ROWDIR) {
      const f32x4* p = reinterpret_cast<const f32x4*>(ab + r * 32 + 16 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 x = p[q];
        fa[4 * q + 0] = x[0]; fa[4 * q + 1] = x[1]; fa[4 * q + 2] = x[2]; fa[4 * q + 3] = x[3];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) fa[s] = ab[(16 * h + s) * 32 + r];
    }
    const size_t krow = (size_t)bc * 32 + 16 * h;
    if constexpr (BROW) {
#pragma unroll
      for (int s = 0; s < 16; ++s) fb[s] = B[(krow + s) * ldb + jld];
    } else {
      const f32x4* p = reinterpret_cast<const f32x4*>(B + (size_t)jld * ldb + krow);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 x = p[q];
        fb[4 * q + 0] = x[0]; fb[4 * q + 1] = x[1]; fb[4 * q + 2] = x[2]; fb[4 * q + 3] = x[3];
      }
    }
  };

  auto mfma16 = [&](const float (&fa)[16], const float (&fb)[16]) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s], fb[s], acc, 0, 0, 0);
  };
  // Two fragment buffers with fixed roles (loop unrolled by 2): block k+1's
  // loads are in flight while block k's MFMAs issue, and no register copy
  // ties the MFMAs to the loads just issued. Prefetches are unconditional
  // (index clamped to the last block; the tail re-reads it and skips the
  // MFMAs), so no branch around a load makes hipcc's counted waits collapse.
  float a0[16], b0[16], a1[16], b1[16];
  const int kl = k1 - 1;
  if (k0 < k1) {
    load_frags(k0, a0, b0);
    settle(a0);
    settle(b0);
  }
  if constexpr ((VAR & 3) == 1) {
    for (int k = k0; k < k1; k += 2) {
      load_frags(min(k + 1, kl), a1, b1);
      mfma16(a0, b0);
      load_frags(min(k + 2, kl), a0, b0);
      if (k + 1 < k1) mfma16(a1, b1);
    }
  } else if constexpr ((VAR & 3) == 2) {
    for (int k = k0; k < k1; ++k) {
      if (k > k0) load_frags(k, a0, b0);
      mfma16(a0, b0);
    }
  } else {
    for (int k = k0; k < k1; ++k) {
      if (k + 1 < k1) load_frags(k + 1, a1, b1);
      mfma16(a0, b0);
#pragma unroll
      for (int s = 0; s < 16; ++s) { a0[s] = a1[s]; b0[s] = b1[s]; }
    }
  }

  if (!jok) return;
  const size_t row0 = (size_t)br * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = row0 + 8 * g + 4 * h + e;
      float* p = CROW ? C + row * ldc + jcol : C + (size_t)jcol * ldc + row;
      *p = epi(acc[4 * g + e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 32 fp32, LDS-staged (ROW blocks, row-major B): the shipped bs = 32
// kernel where the layout allows it.
//
// Fragment-shaped loads straight to VGPRs (the kernel above: per block and
// wave 4 A loads touching 32 rows x 32 B and 16 B loads touching 2 rows each)
// cap that kernel at ~41 % of the MFMA peak even when every operand is
// L2-resident (tools/bsr_micro.py: hot / warm / cold B panels all 64-65
// TFLOP/s; MFMA-only 105). Here a workgroup (4 waves, 128 output columns)
// copies each block's A (4 KB) and B panel (32 rows x 512 B) into LDS with
// global_load_lds_dwordx4 — whole 128-B lines, 20 wave-instructions per block
// instead of 80, no VGPRs — D - 1 blocks ahead, then reads its fragments with
// ds_read_b128 (A, XOR-swizzled 16-B chunks, conflict-free) and ds_read_b32
// (B, 32 consecutive columns per half-wave, conflict-free).
//
// Per block k (stage k % D): wait for this wave's copies of block k (counted
// vmcnt), raw s_barrier (every wave's copies landed and every wave is done
// with stage (k-1) % D), issue the copies of block k + D - 1 into that stage
// (index clamped to the row's last block so every iteration issues the same
// count), then 4 + 16 LDS reads and 16 MFMAs.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* gbl_void_t;

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4]<<14)
constexpr int waitcnt_vm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }
// vmcnt(n) and lgkmcnt(0): also retires this wave's LDS writes before a barrier.
constexpr int waitcnt_vm_lgkm0(int n) { return (n & 15) | (7 << 4) | ((n >> 4) << 14); }

// Fused-hybrid epilogue (spmm_hybrid_csrmm_f32). The MFMA tile
// (32 rows x 128 columns, raw sums) goes to LDS; then the 4 waves split the
// block row's 32 rows into contiguous ranges balanced on rows + remainder nnz
// (a merge-path cut over the 33 row pointers, one ballot per wave). A wave
// walks its rows with wave-uniform (scalar) colind/val loads, lanes across the
// 128 columns (one float2 of each B row per lane, 512 B per wave-instruction),
// HB (24) entries in flight per batch, one sequential FMA chain per element in CSR
// order, and writes each row once:
//   C = epi(tile, alpha, beta, C) + alpha * remainder
// which is the two-launch result (BSR kernel, then the CSR kernel with
// beta = 1) bit for bit on every row the CSR kernel keeps in one wave.
// The remainder's HBM gathers of one workgroup overlap other workgroups' MFMA
// phases on the same CU.
constexpr int kHybTs = 136;  // tile row stride (floats): the two half-waves' rows
                             // land 32 banks apart when the tile is written
template <int D, int kHybBatch, bool PAIR = false>
__device__ __forceinline__ void hyb_remainder(float* smem, const f32x16& acc, const f32x16& acc1,
                                              int br, int jt,
                                              int n, const int* __restrict__ rrp,
                                              const int* __restrict__ rci,
                                              const float* __restrict__ rv, int m,
                                              const float* __restrict__ B, int ldb, float alpha,
                                              float beta, float* __restrict__ C, int ldc) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  __syncthreads();  // every wave is done with the stages (copies drained before)
  if constexpr (!PAIR) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) smem[(8 * g + 4 * h + e) * kHybTs + 32 * wv + r] = acc[4 * g + e];
  } else {
    // wave pair (2c, 2c+1) holds the two k halves of columns 64c .. 64c+63
    const int kh = wv & 1, c0 = 64 * (wv >> 1) + r;
    if (kh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          smem[(8 * g + 4 * h + e) * kHybTs + c0] = acc[4 * g + e];
          smem[(8 * g + 4 * h + e) * kHybTs + c0 + 32] = acc1[4 * g + e];
        }
    __syncthreads();
    if (!kh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          smem[(8 * g + 4 * h + e) * kHybTs + c0] += acc[4 * g + e];
          smem[(8 * g + 4 * h + e) * kHybTs + c0 + 32] += acc1[4 * g + e];
        }
  }
  __syncthreads();

  const int R0 = br * 32;
  // lane i (0..32) holds the row pointer of local row i (rows >= m: empty)
  const int rpv = rrp[min(R0 + min(lane, 32), m)];
  const int s0 = __builtin_amdgcn_readlane(rpv, 0);
  const int tot = __builtin_amdgcn_readlane(rpv, 32) - s0;
  const int pos = rpv - s0 + lane;  // merge-path coordinate of row i's start
  auto cut = [&](int w) -> int {
    const int t = (int)(((long long)(tot + 32) * w) / 4);
    return __builtin_popcountll(__ballot(lane <= 32 && pos < t));
  };
  const int i0 = cut(wv), i1 = wv == 3 ? 32 : cut(wv + 1);
  const int j = jt + 2 * lane;
  const bool jok = j < n;
  const int jl = jok ? j : 0;
  // The wave's entries [p, pend) as one stream across its rows, kHybBatch
  // gathers in flight per step (rows average a few entries on power-law
  // graphs, so per-row batches would serialise on latency); a row is written
  // when the stream passes its end.
  int i = i0;
  int next = __builtin_amdgcn_readlane(rpv, i0 + 1);
  float ax = 0.f, ay = 0.f;
  auto flush = [&]() {
    if (jok) {
      const float2 t = *reinterpret_cast<const float2*>(smem + i * kHybTs + 2 * lane);
      float* out = C + (size_t)(R0 + i) * ldc + j;
      float2 o;
      o.x = epi(t.x, alpha, beta, out) + alpha * ax;
      o.y = epi(t.y, alpha, beta, out + 1) + alpha * ay;
      *reinterpret_cast<float2*>(out) = o;
    }
    ax = ay = 0.f;
    ++i;
    next = __builtin_amdgcn_readlane(rpv, min(i + 1, 32));
  };
  int p = __builtin_amdgcn_readlane(rpv, i0);
  const int pend = __builtin_amdgcn_readlane(rpv, i1);
  while (p < pend) {
    const int nb = min(kHybBatch, pend - p);
    float2 b[kHybBatch];
    float a[kHybBatch];
#pragma unroll
    for (int u = 0; u < kHybBatch; ++u) {
      const int q = min(p + u, pend - 1);  // clamped: same count every step
      a[u] = rv[q];
      b[u] = *reinterpret_cast<const float2*>(B + (size_t)rci[q] * ldb + jl);
    }
#pragma unroll
    for (int u = 0; u < kHybBatch; ++u) {
      if (u < nb) {
        while (i < i1 && p + u >= next) flush();
        ax = __builtin_fmaf(a[u], b[u].x, ax);
        ay = __builtin_fmaf(a[u], b[u].y, ay);
      }
    }
    p += nb;
  }
  while (i < i1) flush();
}

// HYB (the fused hybrid, §4a): after the block loop the workgroup adds its
// 32 rows' CSR remainder (rrp/rci/rv, m rows) — see hyb_remainder below.
// Only CROW is instantiated with HYB.
// XM: block-row order across the 8 XCDs (dispatch puts workgroup b on XCD
// b % 8). 0 = as dispatched; 1 = each XCD a contiguous eighth (neighbouring
// block rows share that XCD's L2); XM >= 2 = chunks of XM block rows dealt
// round-robin to the XCDs (L2 locality inside a chunk, and a heavy region of
// the matrix spread over all XCDs instead of landing on one).
__device__ __forceinline__ int xcd_block_row(int b, int mb, int xm) {
  if (xm == 1) {
    const int q = mb / 8, rem = mb % 8, x = b % 8, i = b / 8;
    return (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + i;
  }
  if (xm >= 2) {
    const int full = mb / (8 * xm) * (8 * xm);
    if (b >= full) return b;
    const int x = b % 8, i = b / 8;
    return ((i / xm) * 8 + x) * xm + i % xm;
  }
  return b;
}

// Split-bf16 products (SPLIT, opt-in: SPMM_HYBRID_SPLIT_BF16). Truncating an
// fp32 x to its top 8 significant bits three times splits it exactly,
// x = hi + mid + lo, each a bf16 (|mid| < 2^-7 |x|, |lo| < 2^-15 |x|). Of the
// nine cross products the six above 2^-22 |a||b| run on
// v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA rate per clock); the three
// dropped ones are below 2^-21 |a||b| together. Per k = 16: 6 bf16 MFMAs of
// 32 cycles in place of 8 fp32 ones of 64.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3_bf16(const float* x, bf16x8& hi, bf16x8& hif, bf16x8& mid,
                                            bf16x8& lo) {
  u32x4 h, hf, m, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const unsigned x0 = __float_as_uint(x[2 * p]), x1 = __float_as_uint(x[2 * p + 1]);
    const bool f0 = (x0 & 0x7f800000u) != 0x7f800000u, f1 = (x1 & 0x7f800000u) != 0x7f800000u;
    // Inf / NaN: hi carries the value (Inf - Inf would make mid and lo NaN)
    const float r0 = f0 ? x[2 * p] - __uint_as_float(x0 & 0xffff0000u) : 0.f;
    const float r1 = f1 ? x[2 * p + 1] - __uint_as_float(x1 & 0xffff0000u) : 0.f;
    const unsigned q0 = __float_as_uint(r0), q1 = __float_as_uint(r1);
    const float l0 = r0 - __uint_as_float(q0 & 0xffff0000u);
    const float l1 = r1 - __uint_as_float(q1 & 0xffff0000u);
    // upper halves of (elem 2p, elem 2p+1) -> one packed bf16 pair, low k first
    h[p] = __builtin_amdgcn_perm(x1, x0, 0x07060302u);
    hf[p] = __builtin_amdgcn_perm(f1 ? x1 : 0u, f0 ? x0 : 0u, 0x07060302u);
    m[p] = __builtin_amdgcn_perm(q1, q0, 0x07060302u);
    l[p] = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
  }
  hi = __builtin_bit_cast(bf16x8, h);
  hif = __builtin_bit_cast(bf16x8, hf);
  mid = __builtin_bit_cast(bf16x8, m);
  lo = __builtin_bit_cast(bf16x8, l);
}

// The six split products of one k range into acc. The high parts meet the
// other operand's mid / lo parts in their finite-only form (hif: Inf / NaN
// lanes zeroed), so a non-finite a meets b only through hi x hi, as an fp32
// product would: Inf * (b_mid = 0) would otherwise add a NaN.
__device__ __forceinline__ f32x16 split_mfma6(const bf16x8& ah, const bf16x8& ahf,
                                              const bf16x8& am, const bf16x8& al,
                                              const bf16x8& bh, const bf16x8& bhf,
                                              const bf16x8& bm, const bf16x8& bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bhf, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahf, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bhf, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahf, bm, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

// HB: remainder gathers in flight per wave in the fused hybrid (HYB).
// PAIR (with SPLIT, row-major C): split-K over wave pairs. Wave w takes k half
// w & 1 of every block for 64 output columns (two tiles), so it splits 8 A
// values per lane per block instead of 16; the pair's partial tiles are added
// through LDS once per block row.
template <bool CROW, int D, int XM, bool HYB = false, int HB = 24, bool SPLIT = false,
          bool PAIR = false>
__global__ __launch_bounds__(256) void bsr32_f32_lds_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, const int* __restrict__ rrp, const int* __restrict__ rci,
    const float* __restrict__ rv, int m, const int* __restrict__ order) {
  constexpr int kStage = 1024 + 32 * 128;  // floats: A block + B panel (20 KB)
  __shared__ __attribute__((aligned(16))) float smem[D * kStage];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, XM);
  const int jt = blockIdx.y * 128;  // first output column of the workgroup
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  if (!HYB && k0 >= k1) {  // empty block row: C = beta * C (alpha * 0)
    const int j = jt + 32 * wv + (lane & 31);
    if (j < n)
      for (int e = 0; e < 16; ++e) {
        const size_t row = (size_t)br * 32 + 2 * e + (lane >> 5);
        float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
        *p = epi(0.f, alpha, beta, p);
      }
    return;
  }

  // Copy sources of this wave: A rows 8w .. 8w+7 (one instruction; lane l ->
  // row 8w + l/8, LDS chunk l%8 holding logical chunk (l%8) ^ swz(row)), and
  // B panel rows 8w .. 8w+7 (four instructions, two rows of 512 B each; the
  // column chunk is clamped so every source stays inside B).
  const int a_row = 8 * wv + (lane >> 3);
  const int a_chunk = (lane & 7) ^ ((a_row >> 1) & 7);
  const int a_src = a_row * 32 + 4 * a_chunk;
  const int b_col = min(jt + 4 * (lane & 31), n - 4);
  const int b_row = 8 * wv + (lane >> 5);
  // bc: the block column of block k (wave-uniform).
  auto issue = [&](int k, int bc, int st) {
    const int kk = min(k, k1 - 1);
    float* stage = smem + st * kStage;
    __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)kk * 1024 + a_src),
                                     (lds_void_t)(stage + 256 * wv), 16, 0, 0);
    const float* bsrc = B + ((size_t)bc * 32 + b_row) * ldb + b_col;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(bsrc + (size_t)(2 * i) * ldb),
                                       (lds_void_t)(stage + 1024 + 128 * (8 * wv + 2 * i)), 16,
                                       0, 0);
  };

  static_assert(!PAIR || (SPLIT && CROW), "PAIR needs SPLIT and row-major C");
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc, acc1;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = acc1[e] = 0.f;
  // Block columns through the readlane cursor: no load per block (a scalar
  // load per block sat right before the copies it feeds), one refill per 64.
  if (!HYB || k0 < k1) {
  ColCursor cc(colind, k0, k1, lane);
#pragma unroll
  for (int d = 0; d < D - 1; ++d) issue(k0 + d, cc.get(min(k0 + d, k1 - 1)), d);

  int st = 0;
  for (int k = k0; k < k1; ++k) {
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(5 * (D - 2)));
    __builtin_amdgcn_s_barrier();
    issue(k + D - 1, cc.get(min(k + D - 1, k1 - 1)), st == 0 ? D - 1 : st - 1);
    const float* stage = smem + st * kStage;
    if constexpr (PAIR) {
      // lane (r, h) element i: k = 16 kh + 8h + i; tiles t = 0, 1 at columns 64 ch + 32 t
      const int kh = wv & 1, ch = wv >> 1;
      float fa8[8], fb0[8], fb1[8];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int pc = (4 * kh + 2 * h + q) ^ ((r >> 1) & 7);
        const f32x4 x = *reinterpret_cast<const f32x4*>(stage + r * 32 + 4 * pc);
        fa8[4 * q] = x[0]; fa8[4 * q + 1] = x[1]; fa8[4 * q + 2] = x[2]; fa8[4 * q + 3] = x[3];
      }
      const float* bp = stage + 1024 + (16 * kh + 8 * h) * 128 + 64 * ch + r;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        fb0[i] = bp[i * 128];
        fb1[i] = bp[i * 128 + 32];
      }
      bf16x8 ah, ahf, am, al, bh, bhf, bm, bl;
      split3_bf16(fa8, ah, ahf, am, al);
      split3_bf16(fb0, bh, bhf, bm, bl);
      acc = split_mfma6(ah, ahf, am, al, bh, bhf, bm, bl, acc);
      split3_bf16(fb1, bh, bhf, bm, bl);
      acc1 = split_mfma6(ah, ahf, am, al, bh, bhf, bm, bl, acc1);
      st = st == D - 1 ? 0 : st + 1;
      continue;
    }
    // A fragment: row r, logical chunks 4h .. 4h+3 (k = 16h + s).
    float fa[16], fb[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pc = (4 * h + q) ^ ((r >> 1) & 7);
      const f32x4 x = *reinterpret_cast<const f32x4*>(stage + r * 32 + 4 * pc);
      fa[4 * q] = x[0]; fa[4 * q + 1] = x[1]; fa[4 * q + 2] = x[2]; fa[4 * q + 3] = x[3];
    }
    const float* bs_ = stage + 1024 + (16 * h) * 128 + 32 * wv + r;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) fb[s2] = bs_[s2 * 128];
    if constexpr (SPLIT) {
      // lane (r, h) element i of MFMA j is k = 16h + 8j + i, for A and B alike
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x8 ah, ahf, am, al, bh, bhf, bm, bl;
        split3_bf16(fa + 8 * j, ah, ahf, am, al);
        split3_bf16(fb + 8 * j, bh, bhf, bm, bl);
        acc = split_mfma6(ah, ahf, am, al, bh, bhf, bm, bl, acc);
      }
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2], fb[s2], acc, 0, 0, 0);
    }
    st = st == D - 1 ? 0 : st + 1;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // drain the clamped tail copies
  }

  if constexpr (HYB) {
    hyb_remainder<D, HB, PAIR>(smem, acc, acc1, br, jt, n, rrp, rci, rv, m, B, ldb, alpha, beta,
                               C, ldc);
    return;
  }
  if constexpr (PAIR) {
    const int kh = wv & 1, c0 = 64 * (wv >> 1) + r;
    __syncthreads();  // every wave is done with the stages (copies drained above)
    if (kh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          smem[(8 * g + 4 * h + e) * kHybTs + c0] = acc[4 * g + e];
          smem[(8 * g + 4 * h + e) * kHybTs + c0 + 32] = acc1[4 * g + e];
        }
    __syncthreads();
    if (kh) return;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int jc = jt + c0 + 32 * t;
      if (jc >= n) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lr = 8 * g + 4 * h + e;
          float* p = C + ((size_t)br * 32 + lr) * ldc + jc;
          *p = epi((t ? acc1 : acc)[4 * g + e] + smem[lr * kHybTs + c0 + 32 * t], alpha, beta, p);
        }
    }
    return;
  }
  const int jcol = jt + 32 * wv + r;
  if (jcol >= n) return;
  const size_t row0 = (size_t)br * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = row0 + 8 * g + 4 * h + e;
      float* p = CROW ? C + row * ldc + jcol : C + (size_t)jcol * ldc + row;
      *p = epi(acc[4 * g + e], alpha, beta, p);
    }
  }
}

// 1 KB of zeros: the B row of the padding entries of a column-stream item (one
// 256-column fp16 row), L2-resident.
__device__ __attribute__((aligned(16))) float g_zero_row[256] = {0.f};

// ---------------------------------------------------------------------------
// bs = 32, column stream (ROW blocks, row-major B): one wave per (block row,
// 128 output columns), no barriers. A block-level kernel keeps four waves in
// step on one block at a time, so every block costs a barrier chain and a B
// stage sized for 32 rows although 73-82 % of the blocks on the stand-ins hold
// one nonzero column (round 1's CM / CM4 kernels). Here a wave
// streams the block row as a sequence of ITEMS of nonzero columns:
//  * A ring (NA slots x 4 KB of LDS): block k + DA is copied by LDS-DMA (4 x
//    global_load_lds_dwordx4, XOR-swizzled 16-B chunks) when the producer
//    reaches block k. Its column mask comes from 8 ds_read2st64_b32 (lane l
//    reads column l % 32 of 16 rows), a masked OR of the 16 values and one
//    ballot: no cross-lane reduction.
//  * An item is two nonzero columns (c0, c1): their A columns are read from
//    the A slot into registers at issue time, their two 512-B B rows loaded
//    into registers (below), and the item issued P steps earlier is consumed:
//    v_mfma_f32_32x32x1_2b_f32 per column and 64-column half. The 2-block
//    form takes one k per MFMA, so a single column costs 2 MFMAs and a pair 4
//    (the 32x32x2 step of a lone column is half zeros).
// Waits: loads and LDS-DMA copies retire in issue order (MI355X_MICROARCH.md
// §vmcnt), so the wave keeps a count of the vector-memory operations it
// issued; each slot records the count at its last load and the wait for it
// is vmcnt(q), q the largest ladder value not above the number of younger
// operations (wait_vm_older). All LDS reads are inline asm that end in
// lgkmcnt(0): their results exist when the compiler sees them, and hipcc puts
// no conservative vmcnt(0) before them.
// Tile columns: MFMA half u (0, 1) block b (lane / 32 of the B operand) holds
// output column 4j + 2b + u of lane j, so a lane's B operands of one row are
// one float2 and its four accumulators of one row are one float4 of C.
// ---------------------------------------------------------------------------
typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// s_waitcnt vmcnt(q), q = the largest value <= y of the ladder
// 0 1 2 3 4 6 8 12 16 24 32 48: retires the operation that has y younger
// vector-memory operations, over-waiting by at most a quarter of y (vmcnt is
// 6 bits: y >= 63 needs no wait). A compare tree in one asm statement: as C,
// hipcc's structurizer turned each leaf into a chain of exec-mask moves.
#define SPMM_VM_LADDER(Y)                                                                     \
  "s_cmp_gt_i32 " Y ", 62\n\t"                                                                \
  "s_cbranch_scc1 20f\n\t"                                                                     \
  "s_cmp_gt_i32 " Y ", 15\n\t"                                                                \
  "s_cbranch_scc1 16f\n\t"                                                                     \
  "s_cmp_gt_i32 " Y ", 7\n\t"                                                                 \
  "s_cbranch_scc1 8f\n\t"                                                                      \
  "s_cmp_gt_i32 " Y ", 3\n\t"                                                                 \
  "s_cbranch_scc1 4f\n\t"                                                                      \
  "s_cmp_gt_i32 " Y ", 1\n\t"                                                                 \
  "s_cbranch_scc1 2f\n\t"                                                                      \
  "s_cmp_gt_i32 " Y ", 0\n\t"                                                                 \
  "s_cbranch_scc1 1f\n\t"                                                                      \
  "s_waitcnt vmcnt(0)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "1:\n\t"                                                                                     \
  "s_waitcnt vmcnt(1)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "2:\n\t"                                                                                     \
  "s_cmp_gt_i32 " Y ", 2\n\t"                                                                 \
  "s_cbranch_scc1 3f\n\t"                                                                      \
  "s_waitcnt vmcnt(2)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "3:\n\t"                                                                                     \
  "s_waitcnt vmcnt(3)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "4:\n\t"                                                                                     \
  "s_cmp_gt_i32 " Y ", 5\n\t"                                                                 \
  "s_cbranch_scc1 6f\n\t"                                                                      \
  "s_waitcnt vmcnt(4)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "6:\n\t"                                                                                     \
  "s_waitcnt vmcnt(6)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "8:\n\t"                                                                                     \
  "s_cmp_gt_i32 " Y ", 11\n\t"                                                                \
  "s_cbranch_scc1 12f\n\t"                                                                     \
  "s_waitcnt vmcnt(8)\n\t"                                                                     \
  "s_branch 20f\n"                                                                              \
  "12:\n\t"                                                                                    \
  "s_waitcnt vmcnt(12)\n\t"                                                                    \
  "s_branch 20f\n"                                                                              \
  "16:\n\t"                                                                                    \
  "s_cmp_gt_i32 " Y ", 31\n\t"                                                                \
  "s_cbranch_scc1 32f\n\t"                                                                     \
  "s_cmp_gt_i32 " Y ", 23\n\t"                                                                \
  "s_cbranch_scc1 24f\n\t"                                                                     \
  "s_waitcnt vmcnt(16)\n\t"                                                                    \
  "s_branch 20f\n"                                                                              \
  "24:\n\t"                                                                                    \
  "s_waitcnt vmcnt(24)\n\t"                                                                    \
  "s_branch 20f\n"                                                                              \
  "32:\n\t"                                                                                    \
  "s_cmp_gt_i32 " Y ", 47\n\t"                                                                \
  "s_cbranch_scc1 48f\n\t"                                                                     \
  "s_waitcnt vmcnt(32)\n\t"                                                                    \
  "s_branch 20f\n"                                                                              \
  "48:\n\t"                                                                                    \
  "s_waitcnt vmcnt(48)\n"                                                                       \
  "20:\n\t"

__device__ __forceinline__ void wait_vm_older(int y) {
  asm volatile(SPMM_VM_LADDER("%0") : : "s"(y) : "scc", "memory");
}

// Segments of long block rows for the bs = 32 column stream (row-major C). A
// wave runs as long as its block row; after a longest-first order the longest
// rows still set the makespan when one of them is a large share of the mean
// load per wave slot (RCM-reordered reddit stand-in: 2,257 blocks in its
// longest row against ~1,100 per slot). Rows longer than L blocks are cut into
// ceil(nb / L) segments of equal length; each segment's wave writes its raw
// 32 x 128 tile to a partial buffer, and seg_fixup_kernel sums a row's
// partials in segment order (deterministic) and applies alpha / beta. One
// workgroup builds everything:
//  * pass 1 (rows in contiguous per-thread chunks, a scan): segment, split-row
//    and partial counts per row in row order, so part bases are fixed by the
//    matrix, not by scheduling;
//  * pass 2: split rows -> splits[] {row, part base, segments}; segments ->
//    segs[] {row, k begin, k end, part or -1} in longest-first order (a
//    counting sort on min(length, 1023) as in block_row_order_kernel; the order
//    inside a bucket only schedules);
//  * entries past the counts are marked empty (row -1): the grids are sized by
//    host bounds (segments <= mb + nnzb / L, split rows <= nnzb / L).
__global__ __launch_bounds__(1024) void seg_build_kernel(int mb, const int* __restrict__ rowptr,
                                                         int L, int split_if, int seg_cap,
                                                         int split_cap, int part_cap,
                                                         int4* __restrict__ segs,
                                                         int4* __restrict__ splits) {
  __shared__ int cnt[1024];
  __shared__ int sseg[1024], ssplit[1024], spart[1024];
  __shared__ int over, maxnb;
  const int t = threadIdx.x;
  const int chunk = (mb + 1023) / 1024;
  const int r0 = min(t * chunk, mb), r1 = min(r0 + chunk, mb);
  if (t == 0) maxnb = 0;
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {
  int nseg = 0, nsplit = 0, npart = 0, mx = 0;
  for (int i = r0; i < r1; ++i) {
    const int nb = rowptr[i + 1] - rowptr[i];
    const int k = nb > L ? (nb + L - 1) / L : 1;
    nseg += k;
    nsplit += k > 1;
    npart += k > 1 ? k : 0;
    mx = max(mx, nb);
  }
  if (pass == 0) atomicMax(&maxnb, mx);
  sseg[t] = nseg;
  ssplit[t] = nsplit;
  spart[t] = npart;
  cnt[t] = 0;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scans
    const int a = t >= off ? sseg[t - off] : 0, b = t >= off ? ssplit[t - off] : 0,
              c = t >= off ? spart[t - off] : 0;
    __syncthreads();
    sseg[t] += a;
    ssplit[t] += b;
    spart[t] += c;
    __syncthreads();
  }
  const int total_seg = sseg[1023], total_split = ssplit[1023];
  // the host sized the lists from the nnzb argument: if the row pointer holds
  // more blocks than that, do not split at all (every row one segment, mb <=
  // seg_cap) rather than write past the lists
  // and split only when the longest row is an outlier: more than split_if
  // blocks (twice the mean load per wave slot); splitting ordinary rows costs
  // more than it balances (reddit stand-in: 2.32 vs 2.02 ms)
  if (t == 0)
    over = total_seg > seg_cap || total_split > split_cap || spart[1023] > part_cap ||
           maxnb <= split_if;
  __syncthreads();
  if (over && pass == 0) {
    L = 0x7fffffff;
    __syncthreads();
    continue;
  }
  int split_at = ssplit[t] - nsplit, part_at = spart[t] - npart;
  // histogram of segment lengths (descending buckets)
  for (int i = r0; i < r1; ++i) {
    const int nb = rowptr[i + 1] - rowptr[i];
    const int k = nb > L ? (nb + L - 1) / L : 1;
    const int len = (nb + k - 1) / k;
    atomicAdd(&cnt[1023 - min(len, 1023)], k);
  }
  __syncthreads();
  const int own = cnt[t];
  for (int off = 1; off < 1024; off <<= 1) {
    const int u = t >= off ? cnt[t - off] : 0;
    __syncthreads();
    cnt[t] += u;
    __syncthreads();
  }
  cnt[t] -= own;
  __syncthreads();
  for (int i = r0; i < r1; ++i) {
    const int kb0 = rowptr[i], nb = rowptr[i + 1] - kb0;
    const int k = nb > L ? (nb + L - 1) / L : 1;
    const int len = (nb + k - 1) / k;
    const int b = 1023 - min(len, 1023);
    if (k > 1) splits[split_at++] = make_int4(i, part_at, k, 0);
    for (int j = 0; j < k; ++j) {
      const int pos = atomicAdd(&cnt[b], 1);
      segs[pos] = make_int4(i, kb0 + min(j * len, nb), kb0 + min((j + 1) * len, nb),
                            k > 1 ? part_at + j : -1);
    }
    if (k > 1) part_at += k;
  }
  for (int i = total_seg + t; i < seg_cap; i += 1024) segs[i] = make_int4(-1, 0, 0, -1);
  for (int i = total_split + t; i < split_cap; i += 1024) splits[i] = make_int4(-1, 0, 0, 0);
  break;
  }
}

// C tile of a split block row = epi(sum of its segments' partial tiles, in
// segment order). Partial tile layout: [part][column tile][32 rows][128].
__global__ __launch_bounds__(256) void seg_fixup_kernel(int n, const int4* __restrict__ splits,
                                                        const float* __restrict__ part, float alpha,
                                                        float beta, float* __restrict__ C, int ldc) {
  const int4 sp = splits[blockIdx.x];
  if (sp.x < 0) return;
  const int tile = blockIdx.y, ntiles = gridDim.y;
  const int c4 = threadIdx.x & 31, r8 = threadIdx.x >> 5;  // 4 columns, rows r8 + 8i
  const int col = tile * 128 + 4 * c4;
  if (col >= n) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r8 + 8 * i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < sp.z; ++j)
      acc += *reinterpret_cast<const f32x4*>(
          part + (((size_t)(sp.y + j) * ntiles + tile) * 32 + r) * 128 + 4 * c4);
    f32x4* p = reinterpret_cast<f32x4*>(C + ((size_t)sp.x * 32 + r) * ldc + col);
    if (beta == 0.f) {
      acc *= alpha;
    } else {
      const f32x4 c = *p;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(beta, c[e], alpha * acc[e]);
    }
    *p = acc;
  }
}

// Analysis for the analysed bs = 32 column stream (spmm_bsr32_analysis_f32): per
// block the mask of its nonzero columns (bit c: a value other than +-0 in column
// c, NaN and inf included, as the column streams' own masks) and, for ROW blocks,
// a column-major copy of the values. One wave per block, four per workgroup.
//  * ROW: lane (j, h) loads row j, columns 16h .. 16h + 15 (four 16-B loads); a
//    ballot per column pair (i, 16 + i) gives both bits; the copy writes column
//    16h + i of every row as one 128-B line per half-wave.
//  * COLUMN: lane L loads floats 16L .. 16L + 15 = column L / 2, half L & 1; one
//    ballot, lanes 2c and 2c + 1 folded into bit c.
__global__ __launch_bounds__(256) void bsr32_analysis_kernel(int nnzb, int rowdir,
                                                             const float* __restrict__ val,
                                                             unsigned* __restrict__ masks,
                                                             float* __restrict__ val_col) {
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
    float* dst = val_col ? val_col + (size_t)k * 1024 : nullptr;  // null: masks only
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = x[i >> 2][i & 3];
      const unsigned long long b = __builtin_amdgcn_ballot_w64((__float_as_uint(v) & 0x7fffffffu) != 0u);
      msk |= ((unsigned)b != 0u ? 1u : 0u) << i;
      msk |= ((unsigned)(b >> 32) != 0u ? 1u : 0u) << (16 + i);
      if (val_col) dst[(16 * h + i) * 32 + j] = v;
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

// The same analysis for bs = 16 fp16 (spmm_bsr16_analysis_f16): one wave per
// kAna16Bpw consecutive blocks (512 B each; the loads of all of them issued before
// the first wait: one block per wave left the kernel latency-bound), lane L holding
// 4 halves of each. ROW: lane (r = L / 4, q = L % 4) holds row r, columns 4q ..
// 4q + 3, and writes them to the column-major copy; COLUMN: lane L holds column
// L / 4, rows 4 (L % 4) .. + 3.
constexpr int kAna16Bpw = 8;

__global__ __launch_bounds__(256) void bsr16_analysis_kernel(int nnzb, int rowdir,
                                                             const uint16_t* __restrict__ val,
                                                             unsigned* __restrict__ masks,
                                                             uint16_t* __restrict__ val_col) {
  const int lane = threadIdx.x & 63;
  const long long k0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * kAna16Bpw;
  if (k0 >= nnzb) return;
  typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
  u16x4 xs[kAna16Bpw];
#pragma unroll
  for (int f = 0; f < kAna16Bpw; ++f) {
    const long long k = min(k0 + f, (long long)nnzb - 1);  // past the end: loaded, not used
    xs[f] = *reinterpret_cast<const u16x4*>(val + (size_t)k * 256 + 4 * lane);
  }
#pragma unroll
  for (int f = 0; f < kAna16Bpw; ++f) {
    const long long k = k0 + f;
    if (k >= nnzb) break;
    const u16x4 x = xs[f];
    unsigned msk = 0;
    if (rowdir) {
      const int r = lane >> 2, q = lane & 3;
      uint16_t* dst = val_col + (size_t)k * 256;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned long long b = __builtin_amdgcn_ballot_w64((x[e] & 0x7fffu) != 0u);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          msk |= ((b & (0x1111111111111111ull << qq)) != 0ull ? 1u : 0u) << (4 * qq + e);
        if (val_col) dst[(4 * q + e) * 16 + r] = x[e];  // null: masks only (the group analysis)
      }
    } else {
      const unsigned long long b = __builtin_amdgcn_ballot_w64(
          ((x[0] | x[1] | x[2] | x[3]) & 0x7fffu) != 0u);
#pragma unroll
      for (int c = 0; c < 16; ++c) msk |= (((b >> (4 * c)) & 15ull) != 0ull ? 1u : 0u) << c;
    }
    if (lane == 0) masks[k] = msk;
  }
}

// Longest-first block-row order for the one-wave-per-block-row kernels (the
// column streams). Their waves run as long as their block rows; when the grid
// is only a few waves per slot deep, dispatching in block-row order leaves a
// tail of long rows started last (reddit stand-in, bs 32: a list-scheduling
// model puts the makespan 55 % above the mean load, 18 % with the longest
// rows first). A counting sort by blocks per row, descending, in one
// workgroup: histogram of min(nnzb_row, 1023) in LDS, a scan, a scatter. The
// order inside a bucket is whatever the atomics give: it only schedules, every
// block row's result is the same in any order.
// With a CSR remainder (crp, the fused hybrid: m rows, 32 per block row) the
// key is (32 x blocks + remainder entries) / 8: a dense block's MFMA work
// weighs about as much as 32 remainder gathers.
// G > 1: i is a group of G block rows (bsr_small_grp_kernel; m = the block rows), keyed by its
// blocks >> gshift.
__device__ __forceinline__ int block_row_key(int i, const int* __restrict__ rowptr,
                                             const int* __restrict__ crp, int m, int sub,
                                             int G = 1, int gshift = 0) {
  if (G > 1) return min((rowptr[min((i + 1) * G, m)] - rowptr[i * G]) >> gshift, 1023);
  // sub: 32-row halves of bs-64 block rows (the SUB column stream), two sub-blocks each
  const int nb = (rowptr[(i >> sub) + 1] - rowptr[i >> sub]) << sub;
  if (!crp) return min(nb, 1023);
  const int rem = crp[min(32 * i + 32, m)] - crp[32 * i];
  return min((32 * nb + rem) >> 3, 1023);
}
__global__ __launch_bounds__(1024) void block_row_order_kernel(int mb, const int* __restrict__ rowptr,
                                                               const int* __restrict__ crp, int m,
                                                               int sub, int* __restrict__ order,
                                                               int G = 1, int gshift = 0) {
  __shared__ int cnt[1024];
  const int t = threadIdx.x;
  cnt[t] = 0;
  __syncthreads();
  for (int i = t; i < mb; i += 1024) atomicAdd(&cnt[1023 - block_row_key(i, rowptr, crp, m, sub, G, gshift)], 1);
  __syncthreads();
  const int own = cnt[t];
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan
    const int u = t >= off ? cnt[t - off] : 0;
    __syncthreads();
    cnt[t] += u;
    __syncthreads();
  }
  cnt[t] -= own;  // exclusive
  __syncthreads();
  for (int i = t; i < mb; i += 1024)
    order[atomicAdd(&cnt[1023 - block_row_key(i, rowptr, crp, m, sub, G, gshift)], 1)] = i;
}

// ---------------------------------------------------------------------------
// bs = 32, column stream with register items (CS2). A round-2 form staged an
// item's two B rows in an LDS ring (8 KB of its 20 KB), which held it to
// eight waves per CU, and read them back with one more LDS round trip per
// item. Here the rows go straight into registers: per item one or two
// global_load_dwordx2 (lane (j, h) columns 4j + 2h, 4j + 2h + 1 of a row:
// the 64 lanes read the 512-B row whole), in a ring of P register slots
// (the loop is unrolled P times). LDS holds only the A ring (12 KB at NA =
// 3), so registers, not LDS, set the occupancy (3 waves per SIMD).
//  * Every vector-memory operation of the loop is counted as before (A
//    copies, B row loads, the block-column chunks), and every wait is the
//    run-time ladder on that count.
//  * The B row loads, the A column reads and the block-column chunk loads are
//    inline asm that does NOT wait: hipcc does not know their registers are
//    in flight. Their destination registers are therefore touched only by
//    other inline asm: the consume step's asm waits (vmcnt ladder, then
//    lgkmcnt(0)) and only then copies them into ordinary registers for the
//    MFMAs. tests/test_isa_waits.py checks on the emitted code that no
//    compiler-generated instruction reads or writes those registers.
//  * Block columns come 64 at a time into one VGPR (lane l: colind[k0 +
//    64c + l], read with v_readlane), the next chunk loaded ahead, so the
//    loop has no scalar loads (an SMEM load in flight would make each
//    lgkmcnt(0) of the LDS reads wait for it too).
// ---------------------------------------------------------------------------
// O32: the B-row loads take the block's panel base in SGPRs and the row
// offset c * ldb * 4 + column offset in the 32-bit VGPR offset (one s_mul and
// one v_add per load instead of a 64-bit address on the scalar unit); needs
// 32 * ldb * 4 < 2^31 (checked by the launcher).
// PK: an item whose block has no second column left takes the first column
// of the next block (its A column from that block's slot, its B row from that
// block's panel), so single-column blocks no longer make half-empty items.
// The first column's A read is complete before the next block's A copy can
// reuse its slot: advancing reads the new block's mask with lgkmcnt(0) before
// it issues that copy (NA = 3: the copy of block k + 3 lands in block k's slot).
// ANT: the A copies are non-temporal (nt). A is read once per column tile and
// never again, so its lines should not displace the B rows that neighbouring
// block rows share in the XCD's L2 (products stand-in 3.15 -> 3.07 ms, reddit
// 2.04 -> 1.93, profiles/r03_var_sweep.jsonl).
// MSK (the analysed form, spmm_bsrmm_analysed_f32): the blocks are column-major
// (COLUMN direction, or the column-major copy spmm_bsr32_analysis_f32 made of ROW
// blocks) and masks[k] holds block k's nonzero columns, computed once per matrix.
// No A ring and no mask reads: per item the wave loads only its nonzero columns'
// A values, one 128-B line per column (lane j: row j), straight into registers
// beside the B rows, and the masks come 64 blocks at a time like the block
// columns. A's bytes fall from the whole block to the nonzero columns (products
// stand-in: 7.5 of 32 columns), and the kernel needs no LDS (row-major C).
// SUB (bs = 64 ROW blocks): a 64 x 64 block is four 32 x 32 sub-blocks with a
// row stride of 64 floats, and the wave of 32-row block row br streams the
// sub-blocks (br & 1, 0) and (br & 1, 1) of every block of bs-64 block row
// br / 2, in that order, as if they were blocks of a bs-32 matrix whose
// block columns are 2 bc and 2 bc + 1: virtual block index v, block v / 2,
// sub-block column v & 1. mb is then the number of 32-row block rows.
// C64 (n <= 64): a 64-column tile. Lane (j, h) loads one float of a B row
// (column 2 j + h: the 64 lanes read 256 B) and each column of an item is ONE
// v_mfma_f32_32x32x1_2b_f32 (block h of the instruction = column 2 j + h)
// instead of two; the second accumulator is not kept. The 128-column tile
// computed 128 columns at n = 64, half of them clamped copies (the reference's
// own sweep at dim 64, benchmark.py:5-8: bs 32 and 64 took the dim-128 time).
// The panel probe's choice (panel_probe_kernel, bsr32_f32_panel_kernel below): the sampled
// blocks hold at least kPanelMin of their 32 columns on average (from kPanelMinBlocks blocks).
constexpr int kPanelSamples = 4096;
constexpr unsigned kPanelMin = 24;
constexpr int kPanelMinBlocks = 1 << 15;
#ifndef SPMM_PANEL_D64
#define SPMM_PANEL_D64 2
#endif
#ifndef SPMM_PANEL_D128
#define SPMM_PANEL_D128 2
#endif
__device__ __forceinline__ bool panel_chosen(const unsigned long long* stat) {
  return stat[1] > 0 && stat[0] >= (unsigned long long)kPanelMin * stat[1];
}

template <bool CROW, int XM, int P, int NA, bool O32 = false, bool PK = false, bool ANT = false,
          bool MSK = false, bool SUB = false, bool C64 = false>
__global__ __launch_bounds__(64) void bsr32_f32_cs2_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, const int* __restrict__ order,
    const int4* __restrict__ segs = nullptr, float* __restrict__ part = nullptr,
    const unsigned* __restrict__ masks = nullptr,
    const unsigned long long* __restrict__ gate = nullptr) {
  static_assert(NA >= 2 && NA <= 4 && P >= 2 && P <= 16, "ring depths");
  // the panel probe chose bsr32_f32_panel_kernel for this matrix (same bits): nothing to do
  if (gate && panel_chosen(gate)) return;
  static_assert(!(SUB && MSK), "the analysed stream is bs 32 only");
  constexpr int DA = NA - 1;  // A blocks in flight ahead of the producer's block
  constexpr int LDA = SUB ? 64 : 32;  // row stride of a (sub-)block's values
  // (column-major C reuses the LDS for a 128 x 36-float tile)
  __shared__ __attribute__((aligned(16)))
  float smem[MSK && CROW ? 4 : (CROW || NA * 1024 >= 128 * 36 ? NA * 1024 : 128 * 36)];
  const int lane = threadIdx.x;
  const int j = lane & 31, h = lane >> 5;
  // a segment of a block row (seg_build_kernel; row-major C only) or a whole row
  int br, k0, k1, pidx = -1;
  if (segs) {
    const int4 sg = segs[blockIdx.x];
    if (sg.x < 0) return;
    br = sg.x;
    k0 = sg.y;
    k1 = sg.z;
    pidx = sg.w;
  } else {
    br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, XM);
    if constexpr (SUB) {  // virtual sub-block indices (above)
      k0 = 2 * rowptr[br >> 1];
      k1 = 2 * rowptr[(br >> 1) + 1];
    } else {
      k0 = rowptr[br];
      k1 = rowptr[br + 1];
    }
  }
  const int jt = blockIdx.y * (C64 ? 64 : 128);
  const unsigned lds_a = (unsigned)reinterpret_cast<uintptr_t>(smem);

  int a_src[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * q + (lane >> 3);
    a_src[q] = r * LDA + 4 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  auto issue_a = [&](int kk, int slot) {
    const float* src = SUB ? val + (size_t)(kk >> 1) * 4096 + (br & 1) * 2048 + (kk & 1) * 32
                           : val + (size_t)kk * 1024;
    float* dst = smem + slot * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(src + a_src[q & 1] + 16 * LDA * (q >> 1)),
                                       (lds_void_t)(dst + 256 * q), 16, 0, ANT ? 2 : 0);
  };
  unsigned moff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    moff[i] = (unsigned)((2 * i + h) * 128 + 16 * ((j >> 2) ^ i) + 4 * (j & 3));
  auto mask_of = [&](int slot) -> unsigned {
    const unsigned base = lds_a + 4096u * (unsigned)slot;
    f32x2 x[8];
    asm volatile(
        "ds_read2st64_b32 %0, %8 offset1:8\n\t"
        "ds_read2st64_b32 %1, %9 offset1:8\n\t"
        "ds_read2st64_b32 %2, %10 offset1:8\n\t"
        "ds_read2st64_b32 %3, %11 offset1:8\n\t"
        "ds_read2st64_b32 %4, %12 offset1:8\n\t"
        "ds_read2st64_b32 %5, %13 offset1:8\n\t"
        "ds_read2st64_b32 %6, %14 offset1:8\n\t"
        "ds_read2st64_b32 %7, %15 offset1:8\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]),
          "=&v"(x[6]), "=&v"(x[7])
        : "v"(base + moff[0]), "v"(base + moff[1]), "v"(base + moff[2]), "v"(base + moff[3]),
          "v"(base + moff[4]), "v"(base + moff[5]), "v"(base + moff[6]), "v"(base + moff[7])
        : "memory");
    unsigned t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      t |= (__float_as_uint(x[i][0]) | __float_as_uint(x[i][1])) & 0x7fffffffu;  // +-0 is zero
    const unsigned long long b = __builtin_amdgcn_ballot_w64(t != 0u);
    return (unsigned)b | (unsigned)(b >> 32);
  };
  const unsigned a_row = (unsigned)(j * 128);
  const int a_sw = (j >> 1) & 7;
  // byte offset of this lane's B-row piece in a row (C64: one float, else two)
  const unsigned boff = C64 ? 4u * (unsigned)min(jt + 2 * j + h, n - 1)
                            : 4u * (unsigned)min(jt + 4 * j + 2 * h, n - 2);
  const size_t ldb4 = (size_t)ldb * 4;
  const unsigned ldb4u = (unsigned)ldb * 4u;

  f32x32 u0, u1;  // MFMA halves u = 0, 1 (output columns 4j + 2b + u)
#pragma unroll
  for (int e = 0; e < 32; ++e) u0[e] = u1[e] = 0.f;

  int nis = 0;  // vector-memory operations issued by this wave
  int ast[DA];  // count at each A block in flight (k+1 .. k+DA)
  int aslot = NA - 1;
  int k = k0 - 1;
  unsigned m = 0;
  bool more = true;
  const char* bblk = reinterpret_cast<const char*>(B);
  int ccur = 0, cnext = 0, cstamp = 0;  // block-column chunks (cnext: in flight)
  unsigned mcur = 0, mnext = 0;         // MSK: the same chunks of the column masks
  const float* ablk = val;              // MSK: the current block's column-major values
  auto load_cols = [&](int kstart) {
    const unsigned off = SUB ? 4u * (unsigned)min((kstart >> 1) + lane, (k1 >> 1) - 1)
                             : 4u * (unsigned)min(kstart + lane, k1 - 1);
    asm volatile("global_load_dword %0, %1, %2" : "=&v"(cnext) : "v"(off), "s"(colind) : "memory");
    if constexpr (MSK) {
      asm volatile("global_load_dword %0, %1, %2" : "=&v"(mnext) : "v"(off), "s"(masks) : "memory");
      ++nis;
    }
    cstamp = ++nis;
  };
  if (k0 < k1) load_cols(k0);
  if constexpr (!MSK) {
#pragma unroll
    for (int d = 0; d < DA; ++d) {
      if (k0 + d < k1) {
        issue_a(k0 + d, d);
        nis += 4;
        ast[d] = nis;
      } else {
        ast[d] = -64;
      }
    }
  }
  typedef typename std::conditional<C64, float, f32x2>::type brow_t;
  int kind[P], stamp[P];
  float ra0[P], ra1[P];    // in flight: asm-only registers
  brow_t rb0[P], rb1[P];   // in flight: asm-only registers
#pragma unroll
  for (int s = 0; s < P; ++s) {
    kind[s] = 0;
    stamp[s] = -64;
    ra0[s] = ra1[s] = 0.f;
    rb0[s] = rb1[s] = brow_t{};
  }

  // next block: its column chunk, A landed, its mask, the copy of block k + DA
  auto advance = [&]() {
    ++k;
    aslot = aslot + 1 == NA ? 0 : aslot + 1;
    const int kr = k - k0;
    constexpr int kChunkV = SUB ? 128 : 64;  // (virtual) blocks per block-column chunk
    if ((kr & (kChunkV - 1)) == 0) {  // next block-column chunk
      if constexpr (MSK)
        asm volatile(SPMM_VM_LADDER("%2") "v_mov_b32 %0, %3\n\tv_mov_b32 %1, %4"
                     : "=&v"(ccur), "=&v"(mcur)
                     : "s"(nis - cstamp), "v"(cnext), "v"(mnext)
                     : "scc", "memory");
      else
        asm volatile(SPMM_VM_LADDER("%1") "v_mov_b32 %0, %2"
                     : "=&v"(ccur)
                     : "s"(nis - cstamp), "v"(cnext)
                     : "scc", "memory");
      if (k + kChunkV < k1) load_cols(k + kChunkV);
    }
    const int bc = SUB ? 2 * __builtin_amdgcn_readlane(ccur, (kr >> 1) & 63) + (kr & 1)
                       : __builtin_amdgcn_readlane(ccur, kr & 63);
    bblk = reinterpret_cast<const char*>(B) + (size_t)bc * 32 * ldb4;
    if constexpr (MSK) {
      m = (unsigned)__builtin_amdgcn_readlane((int)mcur, kr & 63);
      ablk = val + (size_t)k * 1024;
      return;
    }
    wait_vm_older(nis - ast[0]);  // A(k) landed
#pragma unroll
    for (int d = 0; d + 1 < DA; ++d) ast[d] = ast[d + 1];
    m = mask_of(aslot);
    if (k + DA < k1) {
      issue_a(k + DA, aslot + DA >= NA ? aslot + DA - NA : aslot + DA);
      nis += 4;
      ast[DA - 1] = nis;
    } else {
      ast[DA - 1] = -64;
    }
  };
  // MSK: this lane's A value of column c of the current block (row j) into r (in flight)
  auto load_acol = [&](float& r, int c) {
    asm volatile("global_load_dword %0, %1, %2"
                 : "=&v"(r)
                 : "v"(4u * (unsigned)(32 * c + j)), "s"(ablk)
                 : "memory");
    ++nis;
  };
  // LDS address of this lane's A value of column c of the current block
  auto acol = [&](int c) -> unsigned {
    return lds_a + 4096u * (unsigned)aslot + a_row + 16u * (unsigned)((c >> 2) ^ a_sw) +
           4u * (unsigned)(c & 3);
  };
  // B row c of the current block's panel into r (in flight: asm-only register)
  auto load_row = [&](brow_t& r, int c) {
    if constexpr (C64 && O32)
      asm volatile("global_load_dword %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff + (unsigned)c * ldb4u), "s"(bblk)
                   : "memory");
    else if constexpr (C64)
      asm volatile("global_load_dword %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff), "s"(bblk + (size_t)c * ldb4)
                   : "memory");
    else if constexpr (O32)
      asm volatile("global_load_dwordx2 %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff + (unsigned)c * ldb4u), "s"(bblk)
                   : "memory");
    else
      asm volatile("global_load_dwordx2 %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff), "s"(bblk + (size_t)c * ldb4)
                   : "memory");
    ++nis;
  };

  for (;;) {
    const bool fin = !more;
#pragma unroll
    for (int s = 0; s < P; ++s) {
      // consume the item issued P steps ago. The asm runs for empty slots too
      // (their count is old: no wait), so on every path the slot's registers
      // are read by it before the produce step below writes them again.
      if constexpr (C64) {
        float b0, b1, a0, a1;
        asm volatile(SPMM_VM_LADDER("%4")
                     "s_waitcnt lgkmcnt(0)\n\t"
                     "v_mov_b32 %0, %5\n\t"
                     "v_mov_b32 %1, %6\n\t"
                     "v_mov_b32 %2, %7\n\t"
                     "v_mov_b32 %3, %8"
                     : "=&v"(b0), "=&v"(b1), "=&v"(a0), "=&v"(a1)
                     : "s"(nis - stamp[s]), "v"(rb0[s]), "v"(rb1[s]), "v"(ra0[s]), "v"(ra1[s])
                     : "scc", "memory");
        if (kind[s]) {
          u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a0, b0, u0, 0, 0, 0);
          if (kind[s] == 2) u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a1, b1, u0, 0, 0, 0);
        }
      } else {
        f32x2 b0, b1;
        float a0, a1;
        asm volatile(SPMM_VM_LADDER("%4")
                     "s_waitcnt lgkmcnt(0)\n\t"
                     "v_mov_b64 %0, %5\n\t"
                     "v_mov_b64 %1, %6\n\t"
                     "v_mov_b32 %2, %7\n\t"
                     "v_mov_b32 %3, %8"
                     : "=&v"(b0), "=&v"(b1), "=&v"(a0), "=&v"(a1)
                     : "s"(nis - stamp[s]), "v"(rb0[s]), "v"(rb1[s]), "v"(ra0[s]), "v"(ra1[s])
                     : "scc", "memory");
        if (kind[s]) {
          u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a0, b0[0], u0, 0, 0, 0);
          u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(a0, b0[1], u1, 0, 0, 0);
          if (kind[s] == 2) {
            u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a1, b1[0], u0, 0, 0, 0);
            u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(a1, b1[1], u1, 0, 0, 0);
          }
        }
      }
      // produce the next item into slot s
      kind[s] = 0;
      if (more) {
        while (m == 0u) {
          if (k + 1 >= k1) {
            more = false;
            break;
          }
          advance();
        }
        if (m != 0u) {
          const int c0 = __builtin_ctz(m);
          m &= m - 1u;
          if constexpr (PK) {
            // first column: A read and B load now, from this block
            if constexpr (MSK)
              load_acol(ra0[s], c0);
            else
              asm volatile("ds_read_b32 %0, %1" : "=&v"(ra0[s]) : "v"(acol(c0)) : "memory");
            load_row(rb0[s], c0);
            kind[s] = 1;
            while (m == 0u && k + 1 < k1) advance();  // pair with the next block's first column
            if (m != 0u) {
              const int c1 = __builtin_ctz(m);
              m &= m - 1u;
              if constexpr (MSK)
                load_acol(ra1[s], c1);
              else
                asm volatile("ds_read_b32 %0, %1" : "=&v"(ra1[s]) : "v"(acol(c1)) : "memory");
              load_row(rb1[s], c1);
              kind[s] = 2;
            }
          } else {
            int c1 = c0;
            if (m != 0u) {
              c1 = __builtin_ctz(m);
              m &= m - 1u;
            }
            if constexpr (MSK) {
              load_acol(ra0[s], c0);
              load_acol(ra1[s], c1);
            } else {
              asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3"
                           : "=&v"(ra0[s]), "=&v"(ra1[s])
                           : "v"(acol(c0)), "v"(acol(c1))
                           : "memory");
            }
            load_row(rb0[s], c0);
            kind[s] = 1;
            if (c1 != c0) {
              load_row(rb1[s], c1);
              kind[s] = 2;
            }
          }
          stamp[s] = nis;
        }
      }
    }
    if constexpr (C64)
      asm volatile("" : "+a"(u0));
    else
      asm volatile("" : "+a"(u0), "+a"(u1));
    if (fin) break;
  }
  // nothing is in flight after the last round; the full wait makes that
  // visible to the register check (tests/test_isa_waits.py)
  if constexpr (C64 && MSK)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+a"(u0) : "v"(cnext), "v"(mnext) : "memory");
  else if constexpr (C64)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+a"(u0) : "v"(cnext) : "memory");
  else if constexpr (MSK)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)"
                 : "+a"(u0), "+a"(u1)
                 : "v"(cnext), "v"(mnext)
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+a"(u0), "+a"(u1) : "v"(cnext) : "memory");

  // Row-major C goes out non-temporal (C is written once and never re-read here: its
  // lines would displace the B rows neighbouring block rows share; products stand-in
  // 3.25 -> 3.15 ms, reddit unchanged, profiles/r06/ab_cs2b.log)
  if constexpr (CROW && C64) {
    // lane (j, h): rows (e & 3) + 8 (e >> 2) + 4 h, columns 2 j (block 0) and 2 j + 1
    const int col = jt + 2 * j;
    if (col >= n) return;
    if (pidx >= 0) {  // a segment of a split row: the raw tile to its partial (128-float rows)
      float* pt = part + ((size_t)pidx * gridDim.y + blockIdx.y) * 32 * 128;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
        *reinterpret_cast<f32x2*>(pt + row * 128 + 2 * j) = f32x2{u0[e], u0[16 + e]};
      }
      return;
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> AGPR read
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      f32x2* p = reinterpret_cast<f32x2*>(C + row * ldc + col);
      f32x2 v;
      asm volatile("v_accvgpr_read_b32 %0, %2\n\t"
                   "v_accvgpr_read_b32 %1, %3"
                   : "=v"(v[0]), "=v"(v[1])
                   : "a"(u0[e]), "a"(u0[16 + e])
                   : "memory");
      if (beta == 0.f) {
        v *= alpha;
      } else {
        const f32x2 c = *p;
#pragma unroll
        for (int i = 0; i < 2; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
      }
      __builtin_nontemporal_store(v, p);
    }
  } else if constexpr (CROW) {
    const int col = jt + 4 * j;
    if (col >= n) return;
    if (pidx >= 0) {  // a segment of a split row: the raw tile to its partial
      float* pt = part + ((size_t)pidx * gridDim.y + blockIdx.y) * 32 * 128;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
        *reinterpret_cast<f32x4*>(pt + row * 128 + 4 * j) = f32x4{u0[e], u1[e], u0[16 + e], u1[16 + e]};
      }
      return;
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> AGPR read
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      f32x4* p = reinterpret_cast<f32x4*>(C + row * ldc + col);
      f32x4 v = {u0[e], u1[e], u0[16 + e], u1[16 + e]};
      {
        // each row's four accumulators read just before its store: hipcc otherwise copies
        // all 64 out of the AGPRs at once, and those 64 VGPRs set the kernel's register
        // count (148: 3 waves per SIMD; the loop itself needs fewer than 60 besides the
        // accumulators). Analysed products 2.14 -> 2.04 ms at 4 waves per SIMD
        // (profiles/r03_analysed_4waves.txt)
        asm volatile("v_accvgpr_read_b32 %0, %4\n\t"
                     "v_accvgpr_read_b32 %1, %5\n\t"
                     "v_accvgpr_read_b32 %2, %6\n\t"
                     "v_accvgpr_read_b32 %3, %7"
                     : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3])
                     : "a"(u0[e]), "a"(u1[e]), "a"(u0[16 + e]), "a"(u1[16 + e])
                     : "memory");
      }
      if (beta == 0.f) {
        v *= alpha;
      } else {
        const f32x4 c = *p;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
      }
      __builtin_nontemporal_store(v, p);
    }
  } else {
    constexpr int kTs = 36;
    float* tile = smem;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      if constexpr (C64) {
        tile[(2 * j) * kTs + row] = u0[e];
        tile[(2 * j + 1) * kTs + row] = u0[16 + e];
      } else {
        tile[(4 * j) * kTs + row] = u0[e];
        tile[(4 * j + 1) * kTs + row] = u1[e];
        tile[(4 * j + 2) * kTs + row] = u0[16 + e];
        tile[(4 * j + 3) * kTs + row] = u1[16 + e];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const size_t row = (size_t)br * 32 + j;
    for (int it = 0; it < (C64 ? 32 : 64); ++it) {
      const int jl = 2 * it + h;
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + j], alpha, beta, p);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 32 PANEL stream (round 6): the column stream's arithmetic for blocks that hold (nearly)
// every column. On the reference sweep's matrices (test_bsrmm.cu: dense U(-1, 1) blocks) the
// column stream spends 25 scalar instructions per nonzero column on its item bookkeeping and
// keeps the MFMA pipe 32-49 % busy (profiles/r06/pmc_cell/). Here one wave per (block row, TW
// output columns) copies each block's A (4 KB) and its whole B panel (32 rows x TW columns) into
// LDS by LDS-DMA, D stages deep (every block issues the same number of copies, so the waits
// are constants), and runs the block's columns in an unrolled loop: per nonzero column c, in
// ascending order, the MFMAs the column stream issues for it (v_mfma_f32_32x32x1_2b_f32, lane
// (j, h) A = row j's value of column c, B = columns 4j + 2h, + 1 of row c; C64: column 2j + h),
// and nothing for an all-zero column. Each output is thus the same chain of fused
// multiply-adds as in bsr32_f32_cs2_kernel, bit for bit, on every matrix; which of the two
// runs is a question of speed only. panel_probe_kernel samples up to kPanelSamples blocks and
// sums their nonzero-column counts (integers: the order of the atomic adds does not matter);
// the panel stream runs when they hold at least kPanelMin of 32 columns on average, and both
// kernels are launched, the unchosen one exiting at its first instruction.
// Each wave takes kPanelPerWave samples, all of their loads issued together; one pair of
// atomic adds per workgroup of four waves (a pair per sample, 8,192 adds on two addresses,
// took 0.1 ms).
constexpr int kPanelPerWave = 4;
// SUB (bs 64): the samples are 32 x 32 sub-blocks (nnzb counts them, four per block).
__global__ __launch_bounds__(256) void panel_probe_kernel(long long nnzb, int ns, int sub,
                                                          const float* __restrict__ val,
                                                          unsigned long long* __restrict__ stat) {
  __shared__ unsigned part[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int i0 = (blockIdx.x * 4 + w) * kPanelPerWave;
  f32x4 x[kPanelPerWave][4];
#pragma unroll
  for (int t = 0; t < kPanelPerWave; ++t) {
    const int i = min(i0 + t, ns - 1);
    const long long k = (long long)(((long double)i + 0.5L) * (long double)nnzb / ns);
    const float* blk = sub ? val + (size_t)(k >> 2) * 4096 + (k & 2) * 1024 + (k & 1) * 32 + j * 64 + 16 * h
                           : val + (size_t)k * 1024 + j * 32 + 16 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[t][q] = *reinterpret_cast<const f32x4*>(blk + 4 * q);
  }
  unsigned cols = 0, cnt = 0;
#pragma unroll
  for (int t = 0; t < kPanelPerWave; ++t) {
    if (i0 + t >= ns) break;
    unsigned msk = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned long long bl =
            __builtin_amdgcn_ballot_w64((__float_as_uint(x[t][q][e]) & 0x7fffffffu) != 0u);
        msk |= ((unsigned)bl != 0u ? 1u : 0u) << (4 * q + e);
        msk |= ((unsigned)(bl >> 32) != 0u ? 1u : 0u) << (16 + 4 * q + e);
      }
    cols += (unsigned)__builtin_popcount(msk);
    ++cnt;
  }
  if (lane == 0) {
    part[w][0] = cols;
    part[w][1] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned c = part[0][0] + part[1][0] + part[2][0] + part[3][0];
    const unsigned t = part[0][1] + part[1][1] + part[2][1] + part[3][1];
    if (t) {
      atomicAdd(&stat[0], (unsigned long long)c);
      atomicAdd(&stat[1], (unsigned long long)t);
    }
  }
}

// SUB (bs 64): as the column stream's SUB form, one wave per 32-row half br of a block row,
// walking the virtual 32 x 32 sub-blocks kk of its row (block kk / 2, column half kk % 2).
template <bool CROW, bool C64, int D, bool SUB = false>
__global__ __launch_bounds__(64) void bsr32_f32_panel_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, const int* __restrict__ order,
    const unsigned long long* __restrict__ stat) {
  constexpr int TW = C64 ? 64 : 128;        // output columns of the wave
  constexpr int kStage = 1024 + 32 * TW;    // floats: A block + B panel
  constexpr int kOps = 4 + 32 * TW / 256;   // copies per block (16 B per lane each)
  static_assert(D >= 2 && (D - 2) * kOps <= 63, "stages");
  __shared__ __attribute__((aligned(16))) float smem[D * kStage];
  if (!panel_chosen(stat)) return;
  const int lane = threadIdx.x;
  const int j = lane & 31, h = lane >> 5;
  const int br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, 32);
  const int jt = blockIdx.y * TW;
  const int k0 = SUB ? 2 * rowptr[br >> 1] : rowptr[br];
  const int k1 = SUB ? 2 * rowptr[(br >> 1) + 1] : rowptr[br + 1];
  const unsigned lds0 = (unsigned)reinterpret_cast<uintptr_t>(smem);
  // A copies: the column stream's swizzled layout (16-B chunk (l & 7) ^ ((r >> 1) & 7) of row r)
  constexpr int LDA = SUB ? 64 : 32;
  int a_src[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * q + (lane >> 3);
    a_src[q] = r * LDA + 4 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  // B panel copies: instruction i covers rows (64 / (TW / 4)) i .. , lane l the 16 B at row
  // RPI i + l / CPR, column chunk l % CPR (clamped inside the row: n >= 4, n % 4 == 0)
  constexpr int CPR = TW / 4, RPI = 64 / CPR;
  const int b_row = lane / CPR;
  const int b_col = min(jt + 4 * (lane % CPR), n - 4);
  auto issue = [&](int k, int st) {
    const int kk = min(k, k1 - 1);
    float* stage = smem + st * kStage;
    const float* src = SUB ? val + (size_t)(kk >> 1) * 4096 + (br & 1) * 2048 + (kk & 1) * 32
                           : val + (size_t)kk * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(src + a_src[q & 1] + 16 * LDA * (q >> 1)),
                                       (lds_void_t)(stage + 256 * q), 16, 0, 2);
    const int bc = SUB ? 2 * colind[kk >> 1] + (kk & 1) : colind[kk];
    const float* bsrc = B + ((size_t)bc * 32 + b_row) * ldb + b_col;
#pragma unroll
    for (int i = 0; i < 32 / RPI; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(bsrc + (size_t)(RPI * i) * ldb),
                                       (lds_void_t)(stage + 1024 + TW * RPI * i), 16, 0, 0);
  };
  unsigned moff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    moff[i] = (unsigned)((2 * i + h) * 128 + 16 * ((j >> 2) ^ i) + 4 * (j & 3));
  const unsigned a_row = (unsigned)(j * 128);
  const int a_sw = (j >> 1) & 7;
  const unsigned boff = C64 ? 4u * (unsigned)(2 * j + h) : 4u * (unsigned)(4 * j + 2 * h);

  f32x32 u0, u1;
#pragma unroll
  for (int e = 0; e < 32; ++e) u0[e] = u1[e] = 0.f;
  if (k0 < k1) {
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issue(k0 + d, d);
    int st = 0;
    for (int k = k0; k < k1; ++k) {
      // block k's copies landed (the D - 2 blocks issued after it may still be in flight);
      // hand-placed: with D = 2 this is the double buffer's full wait, block k + 1's copies
      // being issued right below, a block of MFMAs ahead of their use
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * kOps) : "memory");
      // refill the stage block k - 1 used (its LDS reads all completed in the last round)
      issue(k + D - 1, st == 0 ? D - 1 : st - 1);
      const unsigned sb = lds0 + 4u * (unsigned)(st * kStage);
      unsigned m;
      {
        f32x2 x[8];
        asm volatile(
            "ds_read2st64_b32 %0, %8 offset1:8\n\t"
            "ds_read2st64_b32 %1, %9 offset1:8\n\t"
            "ds_read2st64_b32 %2, %10 offset1:8\n\t"
            "ds_read2st64_b32 %3, %11 offset1:8\n\t"
            "ds_read2st64_b32 %4, %12 offset1:8\n\t"
            "ds_read2st64_b32 %5, %13 offset1:8\n\t"
            "ds_read2st64_b32 %6, %14 offset1:8\n\t"
            "ds_read2st64_b32 %7, %15 offset1:8\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]),
              "=&v"(x[6]), "=&v"(x[7])
            : "v"(sb + moff[0]), "v"(sb + moff[1]), "v"(sb + moff[2]), "v"(sb + moff[3]),
              "v"(sb + moff[4]), "v"(sb + moff[5]), "v"(sb + moff[6]), "v"(sb + moff[7])
            : "memory");
        unsigned t = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          t |= (__float_as_uint(x[i][0]) | __float_as_uint(x[i][1])) & 0x7fffffffu;
        const unsigned long long bl = __builtin_amdgcn_ballot_w64(t != 0u);
        m = (unsigned)bl | (unsigned)(bl >> 32);
      }
      // the block's columns, 8 at a time: their A values and B rows read, then the MFMAs of
      // the nonzero ones in ascending order
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float a[8];
        typedef typename std::conditional<C64, float, f32x2>::type brow_t;
        brow_t b[8];
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) {
          const int c = 8 * g + c8;
          const unsigned aaddr = sb + a_row + 16u * (unsigned)((c >> 2) ^ a_sw) + 4u * (unsigned)(c & 3);
          const unsigned baddr = sb + 4096u + (unsigned)(c * TW * 4) + boff;
          if constexpr (C64)
            asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3"
                         : "=&v"(a[c8]), "=&v"(b[c8]) : "v"(aaddr), "v"(baddr) : "memory");
          else
            asm volatile("ds_read_b32 %0, %2\n\tds_read_b64 %1, %3"
                         : "=&v"(a[c8]), "=&v"(b[c8]) : "v"(aaddr), "v"(baddr) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) {
          if ((m >> (8 * g + c8)) & 1u) {
            if constexpr (C64) {
              u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a[c8], b[c8], u0, 0, 0, 0);
            } else {
              u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a[c8], b[c8][0], u0, 0, 0, 0);
              u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(a[c8], b[c8][1], u1, 0, 0, 0);
            }
          }
        }
      }
      st = st == D - 1 ? 0 : st + 1;
    }
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // drain the clamped tail copies
  }
  if constexpr (CROW) {
    const int col = jt + (C64 ? 2 : 4) * j;
    if (col >= n) return;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if constexpr (C64) {
        f32x2* p = reinterpret_cast<f32x2*>(C + row * ldc + col);
        f32x2 v = {u0[e], u0[16 + e]};
        if (beta == 0.f) {
          v *= alpha;
        } else {
          const f32x2 c = *p;
#pragma unroll
          for (int i = 0; i < 2; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
        }
        __builtin_nontemporal_store(v, p);
      } else {
        f32x4* p = reinterpret_cast<f32x4*>(C + row * ldc + col);
        f32x4 v = {u0[e], u1[e], u0[16 + e], u1[16 + e]};
        if (beta == 0.f) {
          v *= alpha;
        } else {
          const f32x4 c = *p;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
        }
        __builtin_nontemporal_store(v, p);
      }
    }
  } else {
    constexpr int kTs = 36;
    float* tile = smem;  // every copy has landed (waited above) and no wave reads the stages
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      if constexpr (C64) {
        tile[(2 * j) * kTs + row] = u0[e];
        tile[(2 * j + 1) * kTs + row] = u0[16 + e];
      } else {
        tile[(4 * j) * kTs + row] = u0[e];
        tile[(4 * j + 1) * kTs + row] = u1[e];
        tile[(4 * j + 2) * kTs + row] = u0[16 + e];
        tile[(4 * j + 3) * kTs + row] = u1[16 + e];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const size_t row = (size_t)br * 32 + j;
    for (int it = 0; it < TW / 2; ++it) {
      const int jl = 2 * it + h;
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + j], alpha, beta, p);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 helpers: fp16 transposed LDS reads, the B-panel row swizzle.
// ---------------------------------------------------------------------------
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// N x ds_read_b64_tr_b16 and their lgkmcnt(0) in one asm statement. The
// builtin (__builtin_amdgcn_ds_read_tr16_b64_v4i16) carries no LDS alias
// information, so hipcc's waitcnt pass put a vmcnt(0) before it whenever an
// LDS-DMA copy was in flight: inside the copy loop that drained the copies of
// the blocks ahead once per block (tools/isa_vmcnt.py, loop_drains). The
// results exist for the compiler only after the wait, so nothing can use them
// early. `a[i]` are LDS byte addresses.
__device__ __forceinline__ void ds_read_tr16_x4(f16x4 (&r)[4], const unsigned (&a)[4]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4\n\tds_read_b64_tr_b16 %1, %5\n\t"
      "ds_read_b64_tr_b16 %2, %6\n\tds_read_b64_tr_b16 %3, %7\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
      : "memory");
}
template <int N>
__device__ __forceinline__ void ds_read_tr16_n(f16x4 (&r)[N], const unsigned (&a)[N]) {
  static_assert(N % 4 == 0, "groups of 4");
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    ds_read_tr16_x4(*reinterpret_cast<f16x4(*)[4]>(&r[i]), *reinterpret_cast<const unsigned(*)[4]>(&a[i]));
  }
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)reinterpret_cast<uintptr_t>(p);
}

template <typename T>
__device__ __forceinline__ int bsr16_swz(int row) {
  return sizeof(T) == 2 ? 2 * (row & 7) : 4 * ((row >> 2) & 1);
}

// ---------------------------------------------------------------------------
// bs = 16, column-masked (CM; ROW blocks, row-major B), fp32 or fp16 A/B: a
// workgroup of 4 waves owns (block row, 256 output columns) and copies each
// block's A (16 x 16, row-major) and B panel (16 rows, 16-B-chunk swizzled)
// into LDS with global_load_lds_dwordx4, one raw barrier per block. fp32:
// v_mfma_f32_16x16x4_f32 with k = 4g + s (a lane's A fragment is one
// ds_read_b128); fp16: v_mfma_f32_16x16x16_f16, the B fragment through
// ds_read_b64_tr_b16. Only B rows of nonzero A columns are fetched (41 % on
// the products stand-in at bs = 16); the rest of the stage is zero-filled
// from g_zero_row. The MFMAs are not skipped (see the loop). Copies per iteration:
// P = 1 (A) + 2 (fp16) or 4 (fp32) (B).
// ---------------------------------------------------------------------------
template <typename T, bool CROW, int D = 2, int DA = D + 3, int WPE = 1, int COLS = 256>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void bsr16_cm_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const T* __restrict__ val, const T* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  constexpr int kEpc = 16 / sizeof(T);             // elements per 16-B chunk
  constexpr int kA = 256 * sizeof(T);              // A block bytes
  constexpr int kRowB = COLS * sizeof(T);          // B panel row bytes (COLS columns)
  constexpr int kTpw = COLS / 64;                  // 16-column tiles per wave
  static_assert(kRowB <= 1024, "one B row per copy instruction at most");
  constexpr int kStB = 16 * kRowB;                 // B stage bytes
  constexpr int kRpi = 1024 / kRowB;               // B rows per copy instruction (1 or 2)
  constexpr int kCpr = kRowB / 16;                 // chunks per B row (64 or 32)
  constexpr int kNB = 4 / kRpi;                    // B copy instructions per wave and block
  constexpr int P = 1 + kNB;
  static_assert(D >= 2 && D <= 4 && DA >= D + 2, "ring depths");
  constexpr int W = (1 + P * (D - 2)) < P * (DA - D - 2) ? 1 + P * (D - 2) : P * (DA - D - 2);
  __shared__ __attribute__((aligned(16))) char smem[DA * kA + D * kStB + 64];
  char* const sa = smem;
  char* const sb = smem + DA * kA;
  int* const part = reinterpret_cast<int*>(smem + DA * kA + D * kStB);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = xcd_block_row(blockIdx.x, mb, 1);  // XCD-contiguous block rows
  const int jt = blockIdx.y * COLS;
  const int wc = wv * (COLS / 4);  // first column of this wave inside the tile
  const int g = lane >> 4, c16 = lane & 15;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  if (k0 >= k1) {
#pragma unroll
    for (int t = 0; t < kTpw; ++t) {
      const int j = jt + wc + 16 * t + c16;
      if (j >= n) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t row = (size_t)br * 16 + 4 * g + e;
        float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
        *p = epi(0.f, alpha, beta, p);
      }
    }
    return;
  }

  // A copy: lanes 0 .. kA/64 - 1 of wave w, 16 B each: rows 4w .. 4w+3.
  const bool a_lane = lane < kA / 64;
  const int a_src = (4 * wv) * 16 + lane * kEpc;
  int b_src[kNB], b_rowi[kNB];
#pragma unroll
  for (int i = 0; i < kNB; ++i) {
    const int row = 4 * wv + i * kRpi + lane / kCpr;
    const int c = (lane % kCpr) ^ bsr16_swz<T>(row);
    b_src[i] = row * ldb + min(jt + c * kEpc, n - kEpc);
    b_rowi[i] = row;
  }
  const T* zsrc = reinterpret_cast<const T*>(g_zero_row) + (lane % kCpr) * kEpc;
  auto wrapA = [](int s) { return s >= DA ? s - DA : s; };
  auto issue_a = [&](int k, int slot) {
    const int kk = min(k, k1 - 1);
    if (a_lane)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)kk * 256 + a_src),
                                       (lds_void_t)(sa + slot * kA + wv * (kA / 4)), 16, 0, 0);
  };
  auto issue_b = [&](int bc, unsigned mask, int slot) {
    const T* bp = B + (size_t)bc * 16 * ldb;
#pragma unroll
    for (int i = 0; i < kNB; ++i) {
      const T* src = ((mask >> b_rowi[i]) & 1u) ? bp + b_src[i] : zsrc;
      __builtin_amdgcn_global_load_lds((gbl_void_t)src,
                                       (lds_void_t)(sb + slot * kStB + (4 * wv + i * kRpi) * kRowB),
                                       16, 0, 0);
    }
  };
  // This wave's 4 rows of the A block in ring slot `slot` -> their column mask
  // (lanes 0 .. 15 hold them: a DPP OR inside the first 16-lane row). A value
  // counts as nonzero unless it is +-0 (NaN / inf count).
  const unsigned sa_lds = (unsigned)reinterpret_cast<uintptr_t>(sa);
  // No branch around the read (lanes past the slot re-read lane l % (kA/64)'s
  // 16 B and are masked after): a divergent branch here made the compiler
  // drain every copy in flight (vmcnt(0)) before the read.
  auto partial = [&](int slot) -> int {
    int nib = 0;
    {
      int4 x;  // inline asm for the same reason as full() below
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(x)
                   : "v"(sa_lds + (unsigned)(slot * kA + wv * (kA / 4) + 16 * (lane & (kA / 64 - 1))))
                   : "memory");
      const int xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (sizeof(T) == 2) {
          nib |= ((xs[e] & 0x7fff) != 0) << (2 * e);
          nib |= ((xs[e] & 0x7fff0000) != 0) << (2 * e + 1);
        } else {
          nib |= ((xs[e] & 0x7fffffff) != 0) << e;
        }
      }
      nib = a_lane ? nib << ((lane * kEpc) & 15) : 0;
    }
    nib |= __builtin_amdgcn_update_dpp(0, nib, 0x128, 0xF, 0xF, false);
    nib |= __builtin_amdgcn_update_dpp(0, nib, 0x124, 0xF, 0xF, false);
    nib |= __builtin_amdgcn_update_dpp(0, nib, 0x122, 0xF, 0xF, false);
    nib |= __builtin_amdgcn_update_dpp(0, nib, 0x121, 0xF, 0xF, false);
    return __builtin_amdgcn_readlane(nib, 0);
  };
  const unsigned part_lds = (unsigned)reinterpret_cast<uintptr_t>(part);
  auto full = [&](int k) -> unsigned {  // inline asm: hipcc fences builtin LDS reads with vmcnt(0)
    int4 p;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(p) : "v"(part_lds + 16u * (unsigned)(k & 3)) : "memory");
    return (unsigned)__builtin_amdgcn_readfirstlane(p.x | p.y | p.z | p.w);
  };

  f32x4 acc[kTpw];
#pragma unroll
  for (int t = 0; t < kTpw; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  ColCursor cc(colind, k0, k1, lane);
#pragma unroll
  for (int d = 0; d < DA - 1; ++d) issue_a(k0 + d, d);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int d = 0; d < D; ++d) part[4 * ((k0 + d) & 3) + wv] = partial(d);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0));
  __builtin_amdgcn_s_barrier();
  unsigned mr[D - 1];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    mr[d] = full(k0 + d);
    issue_b(cc.get(min(k0 + d, k1 - 1)), mr[d], d);
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(W < kNB * (D - 2) ? W : kNB * (D - 2)));

  int sA = 0, sB = 0;
  for (int k = k0; k < k1; ++k) {
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(W));
    __builtin_amdgcn_s_barrier();
    const unsigned mnew = full(k + D - 1);
    issue_b(cc.get(min(k + D - 1, k1 - 1)), mnew, sB == 0 ? D - 1 : sB - 1);
    part[4 * ((k + D) & 3) + wv] = partial(wrapA(sA + D));
    issue_a(k + DA - 1, sA == 0 ? DA - 1 : sA - 1);
    const unsigned m = mr[0];
    const char* stage = sa + sA * kA;
    const char* bpan = sb + sB * kStB;
    // MFMAs unconditional: at bs = 16 most blocks use every fp32 k step (each
    // covers 4 columns) and fp16 takes the block in one step, and branching
    // around them made the compiler move the accumulators through VGPRs.
    (void)m;
    if constexpr (sizeof(T) == 2) {
      const f16x4 fa = *reinterpret_cast<const f16x4*>(stage + c16 * 32 + 8 * g);
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int row = 4 * g + q;
      unsigned ad[kTpw];
      f16x4 fb[kTpw];
#pragma unroll
      for (int t = 0; t < kTpw; ++t) {
        const int col = wc + 16 * t + 4 * p;
        ad[t] = lds_addr(bpan + row * kRowB + (((col >> 3) ^ bsr16_swz<T>(row)) << 4) + (col & 7) * 2);
      }
      ds_read_tr16_n(fb, ad);
#pragma unroll
      for (int t = 0; t < kTpw; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa, fb[t], acc[t], 0, 0, 0);
    } else {
      const f32x4 fa = *reinterpret_cast<const f32x4*>(stage + c16 * 64 + 16 * g);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int row = 4 * g + s2;
#pragma unroll
        for (int t = 0; t < kTpw; ++t) {
          const int col = wc + 16 * t + c16;
          const int off = row * kRowB + (((col >> 2) ^ bsr16_swz<T>(row)) << 4) + (col & 3) * 4;
          const float fb = *reinterpret_cast<const float*>(bpan + off);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s2], fb, acc[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int d = 0; d < D - 2; ++d) mr[d] = mr[d + 1];
    mr[D - 2] = mnew;
    sA = wrapA(sA + 1);
    sB = sB == D - 1 ? 0 : sB + 1;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));

  if constexpr (!CROW) {
    // Column-major C: the 16 x COLS tile through LDS, then 4 whole 64-B column
    // segments per store instruction.
    constexpr int kTs = 16;  // floats per tile column
    static_assert(COLS * kTs * 4 <= DA * kA + D * kStB, "tile fits the rings");
    float* tile = reinterpret_cast<float*>(smem);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kTpw; ++t)
      *reinterpret_cast<f32x4*>(tile + (wc + 16 * t + c16) * kTs + 4 * g) = acc[t];
    __syncthreads();
    const size_t row = (size_t)br * 16 + c16;
#pragma unroll 4
    for (int it = 0; it < COLS / 16; ++it) {
      const int jl = 4 * (4 * it + wv) + g;  // local column
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + c16], alpha, beta, p);
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < kTpw; ++t) {
    const int j = jt + wc + 16 * t + c16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16, column stream (CS16; ROW blocks, row-major B). bsr16_cm_kernel
// keeps four waves in step on one block at a time: a barrier per block, and a
// 16-row B stage per block although most of a block's columns are empty (59 %
// on the products stand-in) and their rows come from the zero row. Here one
// wave owns (block row, 256 output columns), no barriers, and streams the
// block row's nonzero columns as ITEMS of 16 packed ACROSS blocks: the k index
// of an item runs over 16 (block, column) pairs, so one
// v_mfma_f32_16x16x16_f16 per 16 output columns takes 16 nonzero columns
// whatever blocks they came from.
// The per-column work runs on the vector unit and the LDS crossbar, not on
// the scalar unit: a first form that picked columns one by one with
// s_ff1 / address arithmetic issued ~590 SALU instructions per item, and the
// one scalar unit per CU, shared by its four SIMDs, bounded it (products
// stand-in 8.4 ms against 5.9 for bsr16_cm_kernel; PMC 2.57 G SALU
// instructions against 1.21 G, profiles/r02_cs16_pmc/).
//  * A ring (NA slots x 512 B): blocks are copied by LDS-DMA two at a time
//    (one global_load_lds_dwordx4, lanes 32-63 the second block), DA + 2
//    blocks ahead of the producer. Reading a block: lane (g, c) reads column
//    c of rows 4g .. 4g + 3 (four ds_read_u16); one ballot and two folds give
//    the column mask (+-0 is zero, anything else, NaN and inf too, counts).
//    The slot is dead after that read.
//  * Pending list, 32 circular entries: lane c < 16 of a block pushes its B
//    row index to entry (ebase + npend + rank) with ds_permute_b32 (rank = one
//    v_bcnt), and every lane (g, c) writes its four A values to the entry's
//    column of the A-fragment buffer (16 rows x 32 entries of fp16 in 72-B
//    rows: the four row groups' writes land in different banks). At 16
//    entries an item is emitted and ebase moves on by 16.
//  * Item stage (P slots x 8 KB), chunk-major: 16-B chunk c (8 columns) of
//    item row r at c * 256 + 16 r. Copy j (global_load_lds_dwordx4) brings
//    chunks 4j .. 4j + 3 of all 16 rows: lane L loads row L & 15, chunk
//    4j + L / 16, so every lane pulls its row index once per item (one
//    ds_bpermute_b32) and each of the 8 copies costs one address add. The
//    transposed reads (ds_read_b64_tr_b16, lane (g, q, p): row 4g + q,
//    columns 16t + 4p ..) are one address plus immediate offsets.
//  * The A fragment (lane (g, r): A[r][k = 4g .. 4g + 3]) is one ds_read_b64
//    of the buffer at emission. Padding (the block row's last item): the zero
//    B row and A values masked to zero in registers, so a padded k adds 0.
//  * The item issued P slots earlier is consumed: a counted wait on its last
//    copy (the run-time vmcnt ladder of bsr32_f32_cs2_kernel: every
//    vector-memory operation of the loop is counted), 16 ds_read_b64_tr_b16
//    under one lgkmcnt wait, 16 MFMAs into 16 accumulator tiles.
// ---------------------------------------------------------------------------
// FLR: copy j (one global_load_lds_dwordx4, 1 KB) brings item rows 2j (lanes 0-31) and
// 2j + 1 (lanes 32-63) whole, so each copy reads 8 whole 128-B lines (a chunk-major form
// read 16 half lines per copy, the other halves one copy later: the L1 / TA work per byte
// was the cost). The stage is row-major (512-B rows); lane k of row R loads
// chunk (k - 2R) & 31, which puts chunk c of row R at 16-B slot (c + 2R) & 31 of its row,
// so the transposed reads are conflict-free and take one address per t (tra).
// ANT: the A copies are non-temporal (nt): each tile's wave reads A from HBM anyway, and
// its lines should not displace the B rows neighbouring block rows share in L2 (products
// stand-in 4.03 -> 3.88 ms, profiles/r03_var_sweep.jsonl).
// MSK (the analysed form, spmm_bsrmm_analysed_f16): the blocks are column-major and
// masks[k] holds block k's nonzero columns (spmm_bsr16_analysis_f16, once per matrix).
// The masks come 64 blocks at a time beside the block columns, so the walk reads no A
// values to find them (no ds_read / ballot round trip), and the A values a block pushes
// (lane (g, c): rows 4g .. 4g + 3 of column c, 8 contiguous bytes) come one pair of
// blocks ahead into registers instead of an LDS ring: 2 KB less LDS per wave.
template <bool CROW, int P, int NA, int DA, int CAP = 48, bool ANT = false, bool CST = false,
          int COLS = 256, bool MSK = false>
__global__ __launch_bounds__(64) void bsr16_f16_cs_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const _Float16* __restrict__ val, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, const int* __restrict__ order,
    const unsigned* __restrict__ masks = nullptr, int ntt = 0) {
  // COLS: output columns per wave (the launcher uses 256). 512 makes a stage row one whole
  // 1-KB B row and serves all 512 columns with one A copy and one walk per block row; 128
  // quarters the stage. Both pass the parity subset and lose on the products stand-in, K =
  // 512: 4.37 ms at 512 (4 waves per CU by LDS) and 4.87 at 128 (4 tiles of A and walk per
  // block row), against 3.77-3.89 at 256 (profiles/r03_cols_per_wave_ab.txt)
  static_assert(COLS == 128 || COLS == 256 || COLS == 512, "columns per wave");
  constexpr int kRowB = COLS * 2;     // bytes per stage row
  constexpr int kCh = COLS / 8;       // 16-B chunks per stage row
  constexpr int kRpc = 1024 / kRowB;  // stage rows per copy (4, 2 or 1)
  constexpr int kCp = 16 / kRpc;      // copies per item
  // the pair copied at block kr (blocks kr + DA + 2, + 3) overwrites blocks
  // kr + DA + 2 - NA, + 3 - NA, which must be read already (< kr)
  static_assert((NA & (NA - 1)) == 0 && DA % 2 == 0 && NA >= DA + 4 && P >= 2 && P <= 6,
                "ring depths");
  // pending-list capacity: 64 entries, or 48 (a smaller A-fragment buffer: 8 waves per CU
  // with NA = 4); a pair of blocks adds at most 32 to at most 15 pending
  static_assert(CAP == 64 || CAP == 48, "pending capacity");
  constexpr int kT = COLS / 16;           // 16-column MFMA tiles per wave
  constexpr int kStage = 16 * COLS * 2;   // one item: 16 B rows x COLS fp16
  // A-fragment buffer row: CAP entries + a dummy entry (index CAP) + pad; 136 / 104 B rows put
  // the four row groups' writes in different banks
  constexpr int kAbRow = CAP == 64 ? 136 : 104;
  constexpr int kAbuf = MSK ? 0 : NA * 512;   // offset of the A-fragment buffer
  constexpr int kStg = kAbuf + 16 * kAbRow;  // offset of the item stages
  constexpr int kLds = kStg + P * kStage;
  static_assert(kLds >= COLS * 16 * 4, "column-major C tile fits");
  static_assert(!CST || kLds >= 16 * (COLS + 4) * 4, "row-major C tile fits");
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int lane = threadIdx.x;
  const int g = lane >> 4, r16 = lane & 15, h = lane >> 5;
  // ntt > 0 (tiles together; TUNING A/B): a 1-D grid in which the ntt column tiles of a
  // block row are consecutive on one XCD (the grouped stream's mapping)
  int bslot = blockIdx.x, tile = blockIdx.y;
  if (ntt > 0) {
    const int L = blockIdx.x, i = L >> 3;
    bslot = (L & 7) + 8 * (i / ntt);
    if (bslot >= mb) return;  // the grid's padding
    tile = i % ntt;
  }
  const int br = order ? order[bslot] : xcd_block_row(bslot, mb, 32);
  const int jt = tile * COLS;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const unsigned lds0 = lds_addr(smem);
  const unsigned abuf = lds0 + kAbuf;

  const size_t ldb2 = (size_t)ldb * 2;
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 2 * (size_t)jt;
  // transposed B reads: lane (g, q = (lane >> 2) & 3, p = lane & 3) reads row R = 4g + q,
  // columns 16t + 4p .. + 3: chunk 2t + p / 2 at byte 8 (p & 1), in slot (chunk + 2R) & 31.
  // Chunk c of row R sits at slot (c + 2R) & 31, so the 32 lanes of a transposed read's lane
  // group (rows 8i .. 8i + 7, chunks 2t, 2t + 1) hit 16 distinct 16-B slots mod 256 B:
  // conflict-free (with c + R, rows R and R + 1 collided on one slot, 2-way: products stand-in
  // 3.79-3.81 -> 3.78-3.80 ms, profiles/r03_swz_ep_lgk_ab.txt)
  constexpr int kSw = 2;
  unsigned boffr[kCp], tra[kT];
#pragma unroll
  for (int j = 0; j < kCp; ++j)
    boffr[j] = 2u * (unsigned)min(
                        jt + 8 * (((lane % kCh) - kSw * (kRpc * j + lane / kCh)) & (kCh - 1)), n - 8);
  {
    const int R = 4 * g + ((lane >> 2) & 3);
#pragma unroll
    for (int t = 0; t < kT; ++t)
      tra[t] = lds0 + kStg + (unsigned)kRowB * R +
               16u * ((2 * t + ((lane & 3) >> 1) + kSw * R) & (kCh - 1)) + 8u * (lane & 1);
  }

  int nis = 0;  // vector-memory operations issued by this wave
  // block columns: 64 at a time in one VGPR (lane l: colind[k0 + 64c + l]), the next chunk in flight
  int ccur = 0, cnext = 0, cstamp = 0;
  unsigned mcur = 0, mnext = 0;  // MSK: the masks of the same chunks
  auto load_cols = [&](int kstart) {
    const unsigned off = 4u * (unsigned)min(kstart + lane, k1 - 1);
    asm volatile("global_load_dword %0, %1, %2" : "=&v"(cnext) : "v"(off), "s"(colind) : "memory");
    if constexpr (MSK) {
      asm volatile("global_load_dword %0, %1, %2" : "=&v"(mnext) : "v"(off), "s"(masks) : "memory");
      ++nis;
    }
    cstamp = ++nis;
  };
  // MSK: the A values of the pair of blocks in flight (an*: asm-only registers) and of the
  // pair being pushed (ac*); lane (g, c): rows 4g .. 4g + 3 of column c
  typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
  u32x2a an0 = {0u, 0u}, an1 = {0u, 0u}, ac0 = {0u, 0u}, ac1 = {0u, 0u};
  int astamp = -64;
  // (each block's base is a 64-bit scalar address: the column-major copy of a large
  // matrix passes 4 GB, which a 32-bit lane offset from val cannot reach; RCM-reordered
  // products, 14.3 M blocks = 7.3 GB, returned wrong values with one)
  const unsigned aoff_lane = 2u * (unsigned)(16 * r16 + 4 * g);
  auto issue_a_reg = [&](int kr_) {  // blocks k0 + kr_, + 1 (clamped)
    const _Float16* b0 = val + (size_t)min(k0 + kr_, k1 - 1) * 256;
    const _Float16* b1 = val + (size_t)min(k0 + kr_ + 1, k1 - 1) * 256;
    asm volatile("global_load_dwordx2 %0, %2, %3\n\t"
                 "global_load_dwordx2 %1, %2, %4"
                 : "=&v"(an0), "=&v"(an1)
                 : "v"(aoff_lane), "s"(b0), "s"(b1)
                 : "memory");
    nis += 2;
    astamp = nis;
  };
  auto issue_a = [&](int kr) {  // blocks k0 + kr, k0 + kr + 1 (kr even) -> slots kr, kr + 1
    const int blk = min(k0 + kr + h, k1 - 1);
    __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)blk * 256 + 8 * (lane & 31)),
                                     (lds_void_t)(smem + (kr & (NA - 1)) * 512), 16, 0,
                                     ANT ? 2 : 0);
    ++nis;
  };
  if (k0 < k1) load_cols(k0);
  int ast[DA / 2 + 1];  // count at each A pair in flight
  if constexpr (MSK) {
    if (k0 < k1) issue_a_reg(0);
  } else {
#pragma unroll
    for (int q = 0; q <= DA / 2; ++q) {
      if (k0 + 2 * q < k1) {
        issue_a(2 * q);
        ast[q] = nis;
      } else {
        ast[q] = -64;
      }
    }
  }

  int kr = 0;  // next block to read, relative to k0 (even)
  const unsigned lowm = (1u << r16) - 1u;
  int prow = 0;  // pending B row indices (lane e: entry e, circular over CAP)
  int npend = 0, ebase = 0;
  // the next two blocks (one A pair): their masks, their columns pushed to the
  // list. One LDS round trip reads both blocks' values, one more pushes both.
  auto advance2 = [&]() {
    if ((kr & 63) == 0) {  // next block-column chunk
      if constexpr (MSK)
        asm volatile(SPMM_VM_LADDER("%2") "v_mov_b32 %0, %3\n\tv_mov_b32 %1, %4"
                     : "=&v"(ccur), "=&v"(mcur)
                     : "s"(nis - cstamp), "v"(cnext), "v"(mnext)
                     : "scc", "memory");
      else
        asm volatile(SPMM_VM_LADDER("%1") "v_mov_b32 %0, %2"
                     : "=&v"(ccur)
                     : "s"(nis - cstamp), "v"(cnext)
                     : "scc", "memory");
      if (k0 + kr + 64 < k1) load_cols(k0 + kr + 64);
    }
    const bool two = k0 + kr + 1 < k1;
    const int bc0 = __builtin_amdgcn_readlane(ccur, kr & 63);
    const int bc1 = __builtin_amdgcn_readlane(ccur, (kr + 1) & 63);
    unsigned m[2];
    unsigned x[8];
    if constexpr (MSK) {
      m[0] = (unsigned)__builtin_amdgcn_readlane((int)mcur, kr & 63) & 0xffffu;
      m[1] = two ? (unsigned)__builtin_amdgcn_readlane((int)mcur, (kr + 1) & 63) & 0xffffu : 0u;
      // pair kr / 2 landed: its A values become current, the next pair goes in flight
      asm volatile(SPMM_VM_LADDER("%4") "v_mov_b64 %0, %2\n\tv_mov_b64 %1, %3"
                   : "=&v"(ac0), "=&v"(ac1)
                   : "v"(an0), "v"(an1), "s"(nis - astamp)
                   : "scc", "memory");
      if (k0 + kr + 2 < k1) issue_a_reg(kr + 2);
      kr += 2;
      if ((m[0] | m[1]) == 0u) return;
      x[0] = ac0[0];
      x[1] = ac0[0] >> 16;
      x[2] = ac0[1];
      x[3] = ac0[1] >> 16;
      x[4] = ac1[0];
      x[5] = ac1[0] >> 16;
      x[6] = ac1[1];
      x[7] = ac1[1] >> 16;
    } else {
    wait_vm_older(nis - ast[0]);  // pair kr / 2 landed
#pragma unroll
    for (int q = 0; q < DA / 2; ++q) ast[q] = ast[q + 1];
    if (k0 + kr + DA + 2 < k1) {
      issue_a(kr + DA + 2);
      ast[DA / 2] = nis;
    } else {
      ast[DA / 2] = -64;
    }
    asm volatile(
        "ds_read_u16 %0, %8\n\t"
        "ds_read_u16 %1, %8 offset:32\n\t"
        "ds_read_u16 %2, %8 offset:64\n\t"
        "ds_read_u16 %3, %8 offset:96\n\t"
        "ds_read_u16 %4, %8 offset:512\n\t"
        "ds_read_u16 %5, %8 offset:544\n\t"
        "ds_read_u16 %6, %8 offset:576\n\t"
        "ds_read_u16 %7, %8 offset:608\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]),
          "=&v"(x[6]), "=&v"(x[7])
        : "v"(lds0 + 512u * (unsigned)(kr & (NA - 1)) + 128u * g + 2u * r16)
        : "memory");
    kr += 2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned long long b =
          __builtin_amdgcn_ballot_w64(((x[4 * u] | x[4 * u + 1] | x[4 * u + 2] | x[4 * u + 3]) & 0x7fffu) != 0u);
      const unsigned w = (unsigned)b | (unsigned)(b >> 32);
      m[u] = (w | (w >> 16)) & 0xffffu;
    }
    if (!two) m[1] = 0u;  // the pair's second copy repeated the last block
    }
    const int cnt0 = __builtin_popcount(m[0]), cnt1 = __builtin_popcount(m[1]);
    if (cnt0 + cnt1 == 0) return;
    // lane c < 16 with bit c set -> entry ebase + npend (+ cnt0) + popcount(mask below c);
    // other lanes -> the entry just before the range (not taken by the merge)
    const int s0 = ebase + npend, s1 = s0 + cnt0;
    int d[2], wa[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool bit = (m[u] >> r16) & 1u;
      const int st = u ? s1 : s0;
      const int e = (st + __builtin_popcount(m[u] & lowm)) % CAP;
      // inactive lanes: an entry the merge below does not take (CAP = 64: the one before
      // the range; CAP = 48: lane 63, which holds no entry)
      d[u] = 4 * (lane < 16 && bit ? e : (CAP == 64 ? (st + 63) & 63 : 63));
      // A values of column r16, rows 4g .. 4g + 3 -> buffer column (entry CAP for empty columns)
      wa[u] = (int)(abuf + 2u * (unsigned)(bit ? e : CAP) + kAbRow * 4u * g);
    }
    int nr0, nr1;
    asm volatile(
        "ds_write_b16 %2, %4\n\t"
        "ds_write_b16 %2, %5 offset:%12\n\t"
        "ds_write_b16 %2, %6 offset:%13\n\t"
        "ds_write_b16 %2, %7 offset:%14\n\t"
        "ds_write_b16 %3, %8\n\t"
        "ds_write_b16 %3, %9 offset:%12\n\t"
        "ds_write_b16 %3, %10 offset:%13\n\t"
        "ds_write_b16 %3, %11 offset:%14\n\t"
        "ds_permute_b32 %0, %15, %17\n\t"
        "ds_permute_b32 %1, %16, %18\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(nr0), "=&v"(nr1)
        : "v"(wa[0]), "v"(wa[1]), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]),
          "v"(x[5]), "v"(x[6]), "v"(x[7]), "n"(kAbRow), "n"(2 * kAbRow), "n"(3 * kAbRow),
          "v"(d[0]), "v"(d[1]), "v"(bc0 * 16 + r16), "v"(bc1 * 16 + r16)
        : "memory");
    const int rel = (lane - s0 + 2 * CAP) % CAP;
    if (lane < CAP) prow = rel < cnt0 ? nr0 : (rel < cnt0 + cnt1 ? nr1 : prow);
    npend += cnt0 + cnt1;
  };

  f32x4 acc[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int kind[P], stamp[P];
  f16x4 fa[P];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    kind[s] = 0;
    stamp[s] = -64;
    fa[s] = f16x4{0, 0, 0, 0};
  }

  bool more = true, blocks = true;
  for (;;) {
    const bool fin = !more;
#pragma unroll
    for (int s = 0; s < P; ++s) {
      // consume the item issued P slots ago (issuing the next item into the stage before
      // the MFMAs, once its fragments are in registers, measured 2.5 % slower)
      if (kind[s]) {
        wait_vm_older(nis - stamp[s]);
#pragma unroll
        for (int hh = 0; hh < (kT + 15) / 16; ++hh) {
          f16x4 fb[16];
          asm volatile(
              "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
              "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
              "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
              "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
              "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
              "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
              "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
              "ds_read_b64_tr_b16 %7, %15 offset:%16\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7])
              : "v"(tra[16 * hh]), "v"(tra[16 * hh + 1]), "v"(tra[16 * hh + 2]),
                "v"(tra[16 * hh + 3]), "v"(tra[16 * hh + 4]), "v"(tra[16 * hh + 5]),
                "v"(tra[16 * hh + 6]), "v"(tra[16 * hh + 7]), "n"(s * kStage)
              : "memory");
          if constexpr (kT >= 16) asm volatile(
              "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
              "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
              "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
              "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
              "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
              "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
              "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
              "ds_read_b64_tr_b16 %7, %15 offset:%16\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[8]), "=&v"(fb[9]), "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]),
                "=&v"(fb[13]), "=&v"(fb[14]), "=&v"(fb[15])
              : "v"(tra[(16 * hh + 8) % kT]), "v"(tra[(16 * hh + 9) % kT]),
                "v"(tra[(16 * hh + 10) % kT]), "v"(tra[(16 * hh + 11) % kT]),
                "v"(tra[(16 * hh + 12) % kT]), "v"(tra[(16 * hh + 13) % kT]),
                "v"(tra[(16 * hh + 14) % kT]), "v"(tra[(16 * hh + 15) % kT]), "n"(s * kStage)
              : "memory");
#pragma unroll
          for (int t = 0; t < (kT < 16 ? kT : 16); ++t)
            acc[16 * hh + t] =
                __builtin_amdgcn_mfma_f32_16x16x16f16(fa[s], fb[t], acc[16 * hh + t], 0, 0, 0);
        }
      }
      // produce the next item into slot s: read blocks until 16 columns are
      // pending or the blocks run out
      kind[s] = 0;
      if (more) {
        while (npend < 16 && blocks) {
          if (k0 + kr >= k1) {
            blocks = false;
            break;
          }
          advance2();
        }
        if (npend == 0) {
          more = false;
        } else {
          const int cnt = min(npend, 16);
          // B rows: lane L -> item row L & 15 (the zero row past cnt); A fragment:
          // lane (g, r) <- A[r][entries 4g .. 4g + 3]; one round trip for both
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          u32x2 y;
          int r;
          asm volatile("ds_bpermute_b32 %0, %2, %3\n\t"
                       "ds_read_b64 %1, %4\n\t"
                       "s_waitcnt lgkmcnt(0)"
                       : "=&v"(r), "=&v"(y)
                       : "v"(4 * ((ebase + r16) % CAP)), "v"(prow),
                         "v"(abuf + kAbRow * (unsigned)r16 + 2u * (unsigned)((ebase + 4 * g) % CAP))
                       : "memory");
          char* const stage = smem + kStg + s * kStage;
          {
            int rw[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) rw[e] = __builtin_amdgcn_readlane(r, e);
            const int sub = lane / (64 / kRpc);  // this lane's row within a copy
#pragma unroll
            for (int j = 0; j < kCp; ++j) {
              const int e = kRpc * j + sub;
              int re = rw[kRpc * j];
#pragma unroll
              for (int u = 1; u < kRpc; ++u) re = sub == u ? rw[kRpc * j + u] : re;
              const char* be = e < cnt ? reinterpret_cast<const char*>(B) + (size_t)re * ldb2 : zrow;
              __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boffr[j]),
                                               (lds_void_t)(stage + 1024 * j), 16, 0, 0);
            }
            nis += kCp;
          }
          unsigned y0 = y[0], y1 = y[1];
          if (cnt < 16) {  // padded entries: stale values (NaN / inf) must not meet the zero rows
            const int e = 4 * g;
            y0 &= (e < cnt ? 0xffffu : 0u) | (e + 1 < cnt ? 0xffff0000u : 0u);
            y1 &= (e + 2 < cnt ? 0xffffu : 0u) | (e + 3 < cnt ? 0xffff0000u : 0u);
          }
          const unsigned u[2] = {y0, y1};
          fa[s] = *reinterpret_cast<const f16x4*>(u);
          kind[s] = 1;
          stamp[s] = nis;
          ebase = (ebase + 16) % CAP;
          npend = npend > 16 ? npend - 16 : 0;
        }
      }
    }
    if (fin) break;
  }
  // nothing is in flight after the last round (a block-column chunk may be: its
  // register stays live until this full wait, which also makes the drain visible to the
  // register check, tests/test_isa_waits.py)
  if constexpr (MSK)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)"
                 :
                 : "v"(cnext), "v"(mnext), "v"(an0), "v"(an1)
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : : "v"(cnext) : "memory");

  if constexpr (!CROW) {
    // column-major C: the 16 x COLS tile through LDS, then 4 whole 64-B column
    // segments per store instruction
    float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int t = 0; t < kT; ++t)
      *reinterpret_cast<f32x4*>(tile + (16 * t + r16) * 16 + 4 * g) = acc[t];
    __builtin_amdgcn_s_waitcnt(0);
    const size_t row = (size_t)br * 16 + r16;
#pragma unroll 4
    for (int it = 0; it < COLS / 4; ++it) {
      const int jl = 4 * it + g;
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * 16 + r16], alpha, beta, p);
      }
    }
    return;
  }
  if constexpr (CST) {
    // row-major C through LDS: the 16 x COLS tile (row pitch COLS + 4 floats: the two
    // half-waves' rows in different banks), then each row as 64 lanes x 16 B (1 KB per
    // store instruction; the register layout stores 4 x 64-B row pieces per instruction:
    // products stand-in 3.91-4.04 -> 3.79-3.90 ms, profiles/r03_epilogue_ab.txt)
    constexpr int kTp = COLS + 4;
    float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int t = 0; t < kT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[(4 * g + e) * kTp + 16 * t + r16] = acc[t][e];
    __builtin_amdgcn_s_waitcnt(0);
    const bool vec = (ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0;
    constexpr int kLpr = COLS >= 256 ? 64 : COLS / 4;  // lanes per row piece
    constexpr int kRpp = 64 / kLpr;                    // rows per store instruction
#pragma unroll
    for (int cc = 0; cc < COLS; cc += 4 * kLpr) {
      const int col = jt + cc + 4 * (lane % kLpr);
      if (col >= n) break;
#pragma unroll 4
      for (int r0 = 0; r0 < 16; r0 += kRpp) {
        const int rr = r0 + lane / kLpr;
        f32x4 v = *reinterpret_cast<const f32x4*>(tile + rr * kTp + cc + 4 * (lane % kLpr));
        float* p = C + ((size_t)br * 16 + rr) * ldc + col;
        if (vec) {
          if (beta == 0.f) {
            v *= alpha;
          } else {
            const f32x4 c = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
          }
          // C written once: non-temporal (3.89 -> 3.80 ms on config 5, profiles/r06/ab_ntc.log)
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) p[i] = epi(v[i], alpha, beta, p + i);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const int j = jt + 16 * t + r16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = C + row * ldc + j;
      __builtin_nontemporal_store(epi(acc[t][e], alpha, beta, p), p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp32 MFMA. Each wave: 16 rows x 64 columns (4 tiles of 16).
// ---------------------------------------------------------------------------
template <bool ROWDIR, bool BROW, bool CROW, int VAR>
__global__ __launch_bounds__(256, (VAR >> 3) ? (VAR >> 3) : 1) void bsr16_f32_mfma_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  constexpr int NT = 4;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = blockIdx.x;
  const int j0 = (blockIdx.y * (blockDim.x >> 6) + wv) * (16 * NT);
  if (j0 >= n) return;
  const int r = lane & 15;
  const int q = lane >> 4;
  int jld[NT];
  bool jok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int jc = j0 + 16 * t + r;
    jok[t] = jc < n;
    jld[t] = jok[t] ? jc : j0;
  }
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  ColCursor cc(colind, k0, k1, lane);
  auto load_frags = [&](int k, float (&fa)[4], float (&fb)[NT][4]) {
    const int bc = (VAR & 4) != 0 ? colind[k] : cc.get(k);
    const float* ab = val + (size_t)k * 256;
    if constexpr (ROWDIR) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(ab + r * 16 + 4 * q);
      fa[0] = x[0]; fa[1] = x[1]; fa[2] = x[2]; fa[3] = x[3];
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) fa[s] = ab[(4 * q + s) * 16 + r];
    }
    const size_t krow = (size_t)bc * 16 + 4 * q;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (BROW) {
#pragma unroll
        for (int s = 0; s < 4; ++s) fb[t][s] = B[(krow + s) * ldb + jld[t]];
      } else {
        const f32x4 x = *reinterpret_cast<const f32x4*>(B + (size_t)jld[t] * ldb + krow);
        fb[t][0] = x[0]; fb[t][1] = x[1]; fb[t][2] = x[2]; fb[t][3] = x[3];
      }
    }
  };

  auto mfma = [&](const float (&fa)[4], const float (&fb)[NT][4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s], fb[t][s], acc[t], 0, 0, 0);
  };
  float a0[4], b0[NT][4];
  if constexpr ((VAR & 3) == 0) {
    // Rotation prefetch: next block loaded under a branch, copied down after use.
    float a1[4], b1[NT][4];
    if (k0 < k1) {
    load_frags(k0, a0, b0);
    settle(a0);
    settle(b0);
  }
    for (int k = k0; k < k1; ++k) {
      if (k + 1 < k1) load_frags(k + 1, a1, b1);
      mfma(a0, b0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a0[s] = a1[s];
#pragma unroll
        for (int t = 0; t < NT; ++t) b0[t][s] = b1[t][s];
      }
    }
  } else if constexpr ((VAR & 3) == 2) {
    // Load-use: latency hidden by occupancy alone (fewest VGPRs).
    for (int k = k0; k < k1; ++k) {
      load_frags(k, a0, b0);
      mfma(a0, b0);
    }
  } else {
    // Fixed-role double buffer, unconditional clamped prefetch (as bs = 32).
    float a1[4], b1[NT][4];
    const int kl = k1 - 1;
    if (k0 < k1) {
    load_frags(k0, a0, b0);
    settle(a0);
    settle(b0);
  }
    for (int k = k0; k < k1; k += 2) {
      load_frags(min(k + 1, kl), a1, b1);
      mfma(a0, b0);
      load_frags(min(k + 2, kl), a0, b0);
      if (k + 1 < k1) mfma(a1, b1);
    }
  }

  const size_t row0 = (size_t)br * 16 + 4 * q;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (!jok[t]) continue;
    const int jc = j0 + 16 * t + r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* p = CROW ? C + (row0 + e) * ldc + jc : C + (size_t)jc * ldc + row0 + e;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16 MFMA (v_mfma_f32_16x16x32_f16): two blocks per instruction.
// Lane quad q: q < 2 -> block b, k = 8q + e; q >= 2 -> block b+1, k = 8(q-2) + e.
// ---------------------------------------------------------------------------
template <bool ROWDIR, bool BROW, bool CROW, int VAR>
__global__ __launch_bounds__(256, (VAR >> 3) ? (VAR >> 3) : 1) void bsr16_f16_mfma_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const _Float16* __restrict__ val, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc) {
  constexpr int NT = 4;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = blockIdx.x;
  const int j0 = (blockIdx.y * (blockDim.x >> 6) + wv) * (16 * NT);
  if (j0 >= n) return;
  const int r = lane & 15;
  const int q = lane >> 4;
  const int half = q >> 1;     // which block of the pair
  const int kq = 8 * (q & 1);  // k offset inside the block
  int jld[NT];
  bool jok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int jc = j0 + 16 * t + r;
    jok[t] = jc < n;
    jld[t] = jok[t] ? jc : j0;
  }
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  ColCursor cc(colind, k0, k1, lane);
  // k: first block of the pair; kk = k + half is this lane's block. When the
  // pair is incomplete the second half re-reads block k and is zeroed at use.
  // k is clamped by the caller to <= k1 - 1; both cursor reads are
  // unconditional (no branch around a load).
  auto load_frags = [&](int k, f16x8& fa, f16x8 (&fb)[NT]) {
    const int k2 = min(k + 1, k1 - 1);
    const int kl = half ? k2 : k;
    int bc;
    if constexpr ((VAR & 4) != 0) {
      bc = colind[kl];  // per-lane load (two addresses per wave)
    } else {
      const int bc0 = cc.get(k);
      const int bc1 = cc.get(k2);
      bc = half ? bc1 : bc0;
    }
    const _Float16* ab = val + (size_t)kl * 256;
    if constexpr (ROWDIR) {
      fa = *reinterpret_cast<const f16x8*>(ab + r * 16 + kq);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) fa[e] = ab[(kq + e) * 16 + r];
    }
    const size_t krow = (size_t)bc * 16 + kq;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (BROW) {
#pragma unroll
        for (int e = 0; e < 8; ++e) fb[t][e] = B[(krow + e) * ldb + jld[t]];
      } else {
        fb[t] = *reinterpret_cast<const f16x8*>(B + (size_t)jld[t] * ldb + krow);
      }
    }
  };

  const f16x8 zero8 = {};
  auto mfma = [&](const f16x8& fa, const f16x8 (&fb)[NT], int k) {
    // Lanes of the missing second block of an odd tail contribute zero.
    const f16x8 fz = (half && k + 1 >= k1) ? zero8 : fa;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fz, fb[t], acc[t], 0, 0, 0);
  };
  f16x8 a0, b0[NT];
  if constexpr ((VAR & 3) == 0) {
    // Rotation prefetch: next pair loaded under a branch, copied down after use.
    f16x8 a1, b1[NT];
    if (k0 < k1) {
    load_frags(k0, a0, b0);
    settle(a0);
    settle(b0);
  }
    for (int k = k0; k < k1; k += 2) {
      if (k + 2 < k1) load_frags(k + 2, a1, b1);
      mfma(a0, b0, k);
      a0 = a1;
#pragma unroll
      for (int t = 0; t < NT; ++t) b0[t] = b1[t];
    }
  } else if constexpr ((VAR & 3) == 2) {
    // Load-use over block pairs: latency hidden by occupancy alone.
    for (int k = k0; k < k1; k += 2) {
      load_frags(k, a0, b0);
      mfma(a0, b0, k);
    }
  } else {
    f16x8 a1, b1[NT];  // fixed-role double buffer over block pairs
    const int kl = k1 - 1;
    if (k0 < k1) {
    load_frags(k0, a0, b0);
    settle(a0);
    settle(b0);
  }
    for (int k = k0; k < k1; k += 4) {
      load_frags(min(k + 2, kl), a1, b1);
      mfma(a0, b0, k);
      load_frags(min(k + 4, kl), a0, b0);
      if (k + 2 < k1) mfma(a1, b1, k + 2);
    }
  }

  const size_t row0 = (size_t)br * 16 + 4 * q;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (!jok[t]) continue;
    const int jc = j0 + 16 * t + r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* p = CROW ? C + (row0 + e) * ldc + jc : C + (size_t)jc * ldc + row0 + e;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// f(integral_constant<S>) for S = 0, 1, ... while it returns true (static slot indices)
template <int... S, class F>
__device__ __forceinline__ void slots_while(std::integer_sequence<int, S...>, F&& f) {
  (void)(f(std::integral_constant<int, S>{}) && ...);
}

// ---------------------------------------------------------------------------
// bs = 2 / 4 / 8, fp32, row-major B: a lane-group VALU kernel
// (rocsparse_bsrmm.h:227-252 sends bs <= 8 to its large-blockdim kernel;
// rocsparse_bsrmm_impl.h:315-389). A bs x bs block feeds too few rows per B row
// for an MFMA tile (8 of 32), and the product is bound by the B-row gathers
// (4 flop per gathered byte at bs 8), so the VALU does the FMAs at a small
// fraction of its rate. One wave per (block row, 64 * VEC columns), four
// independent waves per workgroup. Per block:
//  * A: lane l < bs^2 holds element l of the block (one coalesced load), its
//    column mask is one ballot, and a(r, c) comes to the FMAs by v_readlane;
//  * B: one gather per block column: the 64 lanes read VEC floats each of row
//    bc * bs + c (a whole 256 / 512-B row piece) by a buffer load from a
//    resource built on the row's address in SGPRs (no 64-bit VALU address per
//    gather); a column whose values are all +-0 gets a resource of zero
//    records, so its load returns zeros without touching memory (round 4 read
//    the zero row from L2: a quarter of the gathers on the reddit stand-in).
//    Every block issues the same bs loads and the compiler's counted waits
//    hold across the pipeline (the column-granular contract of include/spmm_hip.h);
//  * pipeline: a ring of R = 4 block slots, A loaded two blocks ahead and the
//    B gathers one block ahead of the FMAs (unrolled R times: static
//    registers, no branch around a load).
// Each output element is one sequential fp32 FMA chain, blocks in order and
// columns in order inside a block: the oracle's bsrmm order bit for bit.
// Workgroups go to the XCDs in chunks of xm (xcd_block_row; 1 = none).
// (Measured and dropped, round 5: the block's values parked in LDS and read back
// as uniform ds_read_b128 broadcasts in place of the v_readlane per value: 2.62
// against 2.06 ms on reddit bs 8. A broadcast read still returns 64 lanes' worth
// of data, so 16-32 of them per block made the LDS the bound.)
// ---------------------------------------------------------------------------
typedef float f32x2v __attribute__((ext_vector_type(2)));

template <int BS, int VEC, bool ROWD, bool CROW>
__global__ __launch_bounds__(256) void bsr_small_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, int xm, const int* __restrict__ dirty = nullptr,
    int gtiles = 0) {
  static_assert(BS == 2 || BS == 4 || BS == 8, "bs 2 / 4 / 8");
  static_assert(VEC == 1 || VEC == 2, "VEC 1 / 2");
  constexpr int E = BS * BS;
  constexpr int R = 4;  // ring slots: A of block k + 2, B of block k + 1, FMAs of block k
  typedef typename std::conditional<VEC == 2, f32x2v, float>::type vec;
  const int lane = threadIdx.x & 63;
  const int wg = xcd_block_row(blockIdx.x, gridDim.x, xm);
  const int br = __builtin_amdgcn_readfirstlane(wg * 4 + (threadIdx.x >> 6));
  if (br >= mb) return;
  // behind bsr_small_grp_kernel: only the 128-column tiles of groups it flagged
  if (dirty && !dirty[(br / (32 / BS)) * gtiles + (int)(blockIdx.y * 64 * VEC) / 128]) return;
  const int col0 = blockIdx.y * 64 * VEC + lane * VEC;
  const bool col_ok = col0 < n;
  const int col_ld = col_ok ? col0 : 0;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const int kl = k1 - 1;
  const int boff = 4 * col_ld;  // the lane's byte offset in a B row

  float acc[BS][VEC];
#pragma unroll
  for (int r = 0; r < BS; ++r)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[r][v] = 0.f;

  float av[R];      // A of a block: lane l < E holds element l
  int bcol[R];      // its block column
  vec x[R][BS];     // its B rows (zero row for empty columns)
  auto load_a = [&](int k, int s) {
    const int kk = min(k, kl);
    av[s] = val[(size_t)kk * E + (lane < E ? lane : 0)];
    bcol[s] = colind[kk];
  };
  auto load_b = [&](int s) {
    const unsigned long long bits =
        __builtin_amdgcn_ballot_w64(lane < E && (__float_as_uint(av[s]) & 0x7fffffffu) != 0u);
    const float* base = B + (size_t)bcol[s] * BS * ldb;  // uniform
#pragma unroll
    for (int c = 0; c < BS; ++c) {
      unsigned long long colbits = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) colbits |= 1ull << (ROWD ? r * BS + c : c * BS + r);
      const bool nz = (bits & colbits) != 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(base + (size_t)c * ldb), 0, nz ? 0x7fffffff : 0, 0x00020000);
      if constexpr (VEC == 2)
        x[s][c] = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b64(rs, boff, 0, 0));
      else
        x[s][c] = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b32(rs, boff, 0, 0));
    }
  };
  auto fma_block = [&](int s) {
#pragma unroll
    for (int c = 0; c < BS; ++c) {
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const float a = __int_as_float(
            __builtin_amdgcn_readlane(__float_as_int(av[s]), ROWD ? r * BS + c : c * BS + r));
        if constexpr (VEC == 1) {
          acc[r][0] = __builtin_fmaf(a, x[s][c], acc[r][0]);
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[r][v] = __builtin_fmaf(a, x[s][c][v], acc[r][v]);
        }
      }
    }
  };

  if (k0 < k1) {
    load_a(k0, 0);
    load_a(k0 + 1, 1);
    load_b(0);
    for (int k = k0; k < k1; k += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        // the loads run for blocks past the row's end too (clamped to its last
        // block): no branch around a load, so the waits stay counted
        load_a(k + u + 2, (u + 2) % R);
        load_b((u + 1) % R);
        if (k + u < k1) fma_block(u);
      }
    }
  }

#pragma unroll
  for (int r = 0; r < BS; ++r) {
    const size_t row = (size_t)br * BS + r;
    if (!col_ok) break;
    if constexpr (CROW) {
      float* p = C + row * ldc + col0;
#pragma unroll
      for (int v = 0; v < VEC; ++v) p[v] = epi(acc[r][v], alpha, beta, p + v);
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float* p = C + (size_t)(col0 + v) * ldc + row;
        p[0] = epi(acc[r][v], alpha, beta, p);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 2 / 4 / 8, fp32, row-major B: the grouped MFMA stream (round 5; the
// drop-in entry's default for these block sizes). bsr_small_kernel gathers a
// B row per (block row, nonzero column) pair: 37.8 M gathers of 512 B on the
// reddit stand-in at bs 8, 19 GB through L2 for 0.12 GB of distinct B, and one
// v_readlane per FMA. Here one wave owns G = 32 / bs adjacent block rows (32
// output rows) x 128 columns and walks the UNION of their block columns in
// ascending order: a B row J * bs + c is loaded once for the whole group and
// multiplied by v_mfma_f32_32x32x1_2b_f32 into all 32 rows at once, the rows of
// block rows that do not hold (J, c) taking a zero A value. On the reddit
// stand-in that is 11.1 M B rows at bs 8 (0.29 of the pairs), 6.2 M at bs 4.
//  * The merge, in batches of 64 candidates (Q = 64 / G per block row, lane =
//    (block row, candidate)): the batch takes, from every block row, its
//    candidates up to the smallest last candidate of any block row that goes on
//    past the batch (so every block column of the batch is complete across the
//    group and the batches come in ascending block-column order), ranks the
//    accepted (J, row) keys in LDS (one broadcast pass over the 64 keys) and
//    writes the batch's union steps: J and, per block row, the block holding J
//    (-1: none). Block columns out of order or repeated inside a row are taken
//    one batch at a time as a prefix of their row, so any input is multiplied
//    whole (in ascending order a batch takes at least one candidate). The next
//    batch's candidates are loaded as soon as a batch is merged.
//  * Per union step (ring of 4 slots, like bsr_small_kernel: A two steps ahead,
//    B one step ahead of the MFMAs): lane (h, j) loads row j % bs of the block its
//    row j's block row holds (bs floats, zero when none); a column c is active
//    when any of the 32 rows has a value other than +-0 in it (bs ballots); the
//    bs B rows go out as 8-B buffer loads (lane (h, j): columns 4j + 2h, + 1, the
//    cs2 layout), an inactive column's from a resource of zero records (no
//    memory traffic); every active column is two MFMAs.
//  * Numerics: a v_mfma_f32_32x32x1 accumulation is one fused multiply-add per
//    output, and a row takes its own block row's (J, c) in ascending order, the
//    other entries adding 0 * b: for sorted block columns each output is the
//    oracle's sequential fp32 FMA chain. The column-granular contract: a tile
//    whose group meets an inf / NaN B value in an active column (one ballot per
//    step) stores nothing and is flagged; bsr_small_kernel, launched behind it
//    on the same stream, recomputes the flagged tiles (its waves of clean tiles
//    exit at once), since 0 * inf would reach the rows of block rows without a
//    value in that column.
// ---------------------------------------------------------------------------
#ifndef SPMM_SGRP_OCC
#define SPMM_SGRP_OCC 1
#endif

#ifndef SPMM_SGRP_PF
#define SPMM_SGRP_PF 1
#endif
#ifndef SPMM_SGRP_LPT
#define SPMM_SGRP_LPT 1
#endif
#ifndef SPMM_SGRP_DB
#define SPMM_SGRP_DB 1
#endif
#ifndef SPMM_SGRP_XM
#define SPMM_SGRP_XM 8
#endif
#ifndef SPMM_SGRP_PROBE
#define SPMM_SGRP_PROBE 1
#endif
// union steps per ring slot at bs 2 / 4 (A/B on the reddit stand-in, profiles/r05c/ab_sp/:
// bs 4 1.50 -> 1.41 ms at 2; bs 2 2.24 -> 2.18 at 2, 2.17 at 4, 2.66 at 8 (220 registers))
#ifndef SPMM_SGRP_SP2
#define SPMM_SGRP_SP2 4
#endif
#ifndef SPMM_SGRP_SP4
#define SPMM_SGRP_SP4 2
#endif

// The grouped stream's choice per matrix (small_grp_probe_kernel, launched before it on the
// same stream). Block rows that share few block columns gain nothing from the union and lose
// to the MFMA's 32 rows; such a matrix is left to bsr_small_kernel whole. Up to 1024 groups
// spread over the matrix are sampled, one wave each: P = 64 / G sample blocks per group, probe
// p being block row (5p + 3) % G's block at position (p + 1/2) / P (a prefix would not do: a
// community's out-of-community columns sort first), searched for in every block row of the
// group by one lane (binary search over its sorted block columns). The mean of 1 / holders
// estimates the union steps per block; the sums go to stat[0..1] as integers (1 / holders in
// units of 1 / 720720, the lcm of 1..16, exact), so the choice does not depend on the order
// the probes' atomic adds land in (a float sum could flip a near-threshold matrix between
// runs). The grouped stream gives the
// whole matrix up past kGiveUp, a little above the break-even of the two kernels on the reddit
// stand-in (bs 8: 2.0 ms for 6.3 M blocks on the lane-group kernel against 1.37 ms for
// 2.75 M union steps, 0.64; bs 4 0.40; bs 2 0.20); a uniform-random pattern (the reference's
// test_bsrmm) sits near 1, reddit at 0.44 / 0.20 / 0.10. Per matrix, not per group: a group
// given up runs its block rows one wave each on the lane-group kernel, and one long group
// there (a hub) made a 0.1-ms tail on reddit; the probes inside the stream itself cost 8-13 %
// (their chains of dependent loads at every wave's start).
constexpr unsigned kProbeUnit = 720720;  // lcm(1..16): 1 / holders for G <= 16 holders
// the grouped stream gives the matrix up (to bsr_small_kernel) past kGiveUp union steps per
// block; also evaluated on the host by spmm_bsr_small_path
__host__ __device__ inline bool small_grp_gives_up(int bs, unsigned long long est,
                                                   unsigned long long nv) {
  const float kGiveUp = bs == 8 ? 0.70f : (bs == 4 ? 0.45f : 0.25f);
  return (double)est > (double)kGiveUp * kProbeUnit * (double)nv;
}

template <int BS>
__global__ __launch_bounds__(64) void small_grp_probe_kernel(int mb, int ngroups,
                                                             const int* __restrict__ rowptr,
                                                             const int* __restrict__ colind,
                                                             unsigned long long* __restrict__ stat) {
  constexpr int G = 32 / BS, P = 64 / G;
  const int g = (int)(((long long)blockIdx.x * ngroups) / gridDim.x);
  const int lane = threadIdx.x, pp = lane / G;
  const int prow = g * G + (pp * 5 + 3) % G, srow = g * G + lane % G;
  const int ps = prow < mb ? rowptr[prow] : 0, pe = prow < mb ? rowptr[prow + 1] : 0;
  const bool pvalid = pe > ps;
  const int pj = pvalid ? colind[ps + (int)(((2LL * pp + 1) * (pe - ps)) / (2 * P))] : -1;
  int lo = srow < mb ? rowptr[srow] : 0;
  const int se = srow < mb ? rowptr[srow + 1] : 0;
  int hi = se;
  while (pvalid && lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (colind[mid] < pj) lo = mid + 1;
    else hi = mid;
  }
  const unsigned long long held = __builtin_amdgcn_ballot_w64(pvalid && lo < se && colind[lo] == pj);
  const unsigned long long pv = __builtin_amdgcn_ballot_w64(pvalid);
  unsigned long long est = 0;  // sum of 720720 / holders: exact
  unsigned nv = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if ((pv >> (p * G)) & 1ull) {
      est += kProbeUnit /
             (unsigned)max(__builtin_popcountll((held >> (p * G)) & ((1ull << G) - 1ull)), 1);
      ++nv;
    }
  }
  if (lane == 0 && nv) {
    atomicAdd(&stat[0], est);
    atomicAdd(&stat[1], (unsigned long long)nv);
  }
}

template <int BS, bool ROWD, bool CROW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SPMM_SGRP_OCC))) void bsr_small_grp_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, int xm, int* __restrict__ dirty,
    const int* __restrict__ order, int nnzb, const unsigned long long* __restrict__ stat) {
  static_assert(BS == 2 || BS == 4 || BS == 8, "bs 2 / 4 / 8");
  constexpr int G = 32 / BS;  // block rows per group: 32 output rows
  constexpr int Q = 64 / G;   // candidates per block row and batch
  constexpr int E = BS * BS;
  constexpr int DB = SPMM_SGRP_DB;  // B rows loaded DB steps ahead of their MFMAs, A DB + 1
  constexpr int R = 4;        // ring slots: A of step s + DB + 1, B of step s + DB, MFMAs of step s
  // union steps per ring slot: at bs 2 / 4 several steps share a slot's bookkeeping (taken in
  // queue order, so every row still adds its (J, c) in ascending order)
  constexpr int SP = BS == 2 ? SPMM_SGRP_SP2 : (BS == 4 ? SPMM_SGRP_SP4 : 1);
  constexpr int SC = SP * BS;  // columns per slot
  constexpr int NQ = 128;     // union-step queue (a batch adds at most 64)
  constexpr int kNone = 0x7fffffff;
  constexpr unsigned long long kSeg = (1ull << Q) - 1;
  __shared__ __attribute__((aligned(16))) unsigned skey[64];  // a batch's keys (J << 5 | row)
  __shared__ unsigned sskey[64];                              // the same, ranked
  __shared__ int sblk[64];                                    // their blocks, ranked
  __shared__ int suj[NQ];                                     // queued step -> block column J
  __shared__ __attribute__((aligned(16))) int suk[NQ * G];    // step, block row -> block (-1)
  __shared__ __attribute__((aligned(16))) float tile[CROW ? 4 : 128 * 36];

  const int lane = threadIdx.x;
  const int j = lane & 31, h = lane >> 5;
  // Groups go to the XCDs in chunks of xm (neighbours share B rows in one L2). With `order`
  // (a shallow grid) the chunks come longest first: order[] ranks them and the grid has
  // nchunks * xm waves, those past the last group exiting at once.
  int g;
  if (order) {
    const int b = blockIdx.x, nch = gridDim.x / xm, full = nch / 8 * 8 * xm;
    const int slot = b < full ? (b / 8 / xm) * 8 + b % 8 : nch / 8 * 8 + (b - full) / xm;
    const int member = b < full ? (b / 8) % xm : (b - full) % xm;
    g = order[slot] * xm + member;
    if (g * G >= mb) return;
  } else {
    g = xcd_block_row(blockIdx.x, gridDim.x, xm);
  }
  // small_grp_probe_kernel's estimate of union steps per block: past kGiveUp the matrix is
  // left to bsr_small_kernel (its block rows share too little)
  {
    if (SPMM_SGRP_PROBE && small_grp_gives_up(BS, stat[0], stat[1])) {
      if (lane == 0) dirty[g * gridDim.y + blockIdx.y] = 1;
      return;
    }
  }
  const int jt = blockIdx.y * 128;
  // merge role: block row lr of the group, candidate lq
  const int lr = lane / Q, lq = lane % Q;
  const int lbr = g * G + lr;
  int lp = lbr < mb ? rowptr[lbr] : 0;
  const int le = lbr < mb ? rowptr[lbr + 1] : 0;
  // step role: output row j is row gi of block row grow of the group
  const int grow = j / BS, gi = j % BS;
  const unsigned boff = 4u * (unsigned)min(jt + 4 * j + 2 * h, n - 2);

  int cj = lp + lq < le ? colind[lp + lq] : kNone;  // the next batch's candidates
  float pf0 = 0.f, pf1 = 0.f;                        // prefetches of the batch's blocks
  int qh = 0, qt = 0;  // union steps queued / taken
  bool done = false;

  // one batch: appends its union steps at qh, returns their number (0: every row done)
  auto merge = [&]() -> int {
    const bool valid = lp + lq < le;
    const bool more = lp + Q < le;  // the row goes on past this batch
    const int lastv = lq == Q - 1 && more ? cj : kNone;
    int cut = kNone;
#pragma unroll
    for (int r = 0; r < G; ++r) cut = min(cut, __builtin_amdgcn_readlane(lastv, r * Q + Q - 1));
    const int prev = __builtin_amdgcn_update_dpp(0, cj, 0x111, 0xf, 0xf, false);  // row_shr:1
    const bool bad = !valid || cj > cut || (lq > 0 && prev >= cj);
    const unsigned long long badm = __builtin_amdgcn_ballot_w64(bad);
    bool acc = ((badm >> (lr * Q)) & kSeg & ((2ull << lq) - 1)) == 0;
    unsigned long long accm = __builtin_amdgcn_ballot_w64(acc);
    if (accm == 0) {  // no prefix below the cut (unsorted input): the first row's head alone
      const unsigned long long heads = __builtin_amdgcn_ballot_w64(valid && lq == 0);
      if (heads == 0) return 0;
      const int f = __builtin_ctzll(heads);
      accm = 1ull << f;
      acc = lane == f;
    }
    const int kblk = lp + lq;
    lp += __builtin_popcountll((accm >> (lr * Q)) & kSeg);
    // the batch's blocks toward L2 now, a batch before their steps load them (the loads
    // are used by the next merge, when they have long landed)
    asm volatile("" ::"v"(pf0), "v"(pf1));
    if (SPMM_SGRP_PF && acc) {
      const float* blk = val + (size_t)kblk * E;
      pf0 = blk[0];
      pf1 = E * 4 > 128 ? blk[32] : 0.f;
    }
    const unsigned key = acc ? ((unsigned)cj << 5) | (unsigned)lr : 0xffffffffu;
    skey[lane] = key;
    __syncthreads();
    int rank = 0;
#pragma unroll
    for (int m = 0; m < 64; m += 4) {
      const uint4 k4 = *reinterpret_cast<const uint4*>(&skey[m]);
      rank += (k4.x < key) + (k4.y < key) + (k4.z < key) + (k4.w < key);
    }
    if (acc) {
      sskey[rank] = key;
      sblk[rank] = kblk;
    }
    __syncthreads();
    const int nacc = __builtin_popcountll(accm);
    const unsigned mkey = lane < nacc ? sskey[lane] : 0u;
    const int mblk = lane < nacc ? sblk[lane] : 0;
    const unsigned pkey = lane > 0 && lane < nacc ? sskey[lane - 1] : 0u;
    const bool first = lane < nacc && (lane == 0 || (pkey >> 5) != (mkey >> 5));
    const unsigned long long fm = __builtin_amdgcn_ballot_w64(first);
    const int q = (qh + __builtin_popcountll(fm & (~0ull >> (63 - lane))) - 1) & (NQ - 1);
    const int nun = __builtin_popcountll(fm);
    if (lane < nun) {
      int* row = &suk[((qh + lane) & (NQ - 1)) * G];
#pragma unroll
      for (int r = 0; r < G; r += 4) *reinterpret_cast<int4*>(row + r) = int4{-1, -1, -1, -1};
    }
    __syncthreads();
    if (lane < nacc) {
      suk[q * G + (int)(mkey & 31u)] = mblk;
      if (first) suj[q] = (int)(mkey >> 5);
    }
    __syncthreads();
    cj = lp + lq < le ? colind[lp + lq] : kNone;
    return nun;
  };

  float ar[R][SC];    // A: row gi of the block row grow's block of each step (zero: none)
  int jr[R][SP];      // the steps' block columns (uniform)
  bool vr[R];         // the slot's first step exists (uniform)
  unsigned act[R];    // active columns (uniform)
  f32x2 bx[R][SC];    // B rows J * bs + c, this lane's two columns
  // A through one buffer resource from the group's first block: a block row without the
  // step's block column reads past the resource's end, zeros without a memory access
  const int kbase = __builtin_amdgcn_readfirstlane(lp);  // lane 0: the group's first block
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(val + (size_t)kbase * E), 0,
      (unsigned)min((long long)(nnzb - kbase) * E * 4, 0x7fffffffLL), 0x00020000);
  const unsigned aoff = 4u * (unsigned)(ROWD ? gi * BS : gi);
  auto load_a = [&](int s) {
#pragma unroll
    for (int p = 0; p < SP; ++p) {
      const bool v = qt < qh;
      const int qi = qt & (NQ - 1);
      const int J = v ? __builtin_amdgcn_readfirstlane(suj[qi]) : 0;
      const int kb = v ? suk[qi * G + grow] : -1;
      qt += v ? 1 : 0;
      if (p == 0) vr[s] = v;
      jr[s][p] = J;
      const unsigned off = kb >= 0 ? (unsigned)(kb - kbase) * (E * 4) + aoff : 0x80000000u;
      float* a = &ar[s][p * BS];
      if constexpr (ROWD && BS == 8) {
        const f32x4 x0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0));
        const f32x4 x1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off + 16, 0, 0));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a[c] = x0[c];
          a[4 + c] = x1[c];
        }
      } else if constexpr (ROWD && BS == 4) {
        const f32x4 x0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0));
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = x0[c];
      } else if constexpr (ROWD) {
        const f32x2 x0 = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rsa, off, 0, 0));
        a[0] = x0[0];
        a[1] = x0[1];
      } else {
#pragma unroll
        for (int c = 0; c < BS; ++c)
          a[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsa, off + 4 * c * BS, 0, 0));
      }
    }
  };
  auto load_b = [&](int s) {
    unsigned m = 0;
#pragma unroll
    for (int c = 0; c < SC; ++c)
      m |= (unsigned)(__builtin_amdgcn_ballot_w64((__float_as_uint(ar[s][c]) & 0x7fffffffu) != 0u) != 0) << c;
    act[s] = m;
    // one resource over each step's bs B rows; an inactive column's offset is past its end,
    // so its load returns zeros without a memory access
#pragma unroll
    for (int p = 0; p < SP; ++p) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(B + (size_t)jr[s][p] * BS * ldb), 0, BS * ldb * 4, 0x00020000);
#pragma unroll
      for (int c = 0; c < BS; ++c)
        bx[s][p * BS + c] = __builtin_bit_cast(
            f32x2, __builtin_amdgcn_raw_buffer_load_b64(
                       rs, boff + ((m >> (p * BS + c)) & 1u ? (unsigned)(c * ldb) * 4u : 0x80000000u), 0, 0));
    }
  };

  f32x32 u0, u1;  // MFMA halves u = 0, 1 (output columns 4j + 2b + u of block b)
#pragma unroll
  for (int e = 0; e < 32; ++e) u0[e] = u1[e] = 0.f;
  auto consume = [&](int s) {
    const unsigned m = act[s];
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      if ((m >> c) & 1u) {
        // the MFMAs' accumulators as values of one use each: hipcc then accumulates in
        // place (dst = srcC) instead of copying 64 registers around every branch
        asm volatile("" : "+a"(u0), "+a"(u1));
        u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(ar[s][c], bx[s][c][0], u0, 0, 0, 0);
        u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(ar[s][c], bx[s][c][1], u1, 0, 0, 0);
      }
    }
  };

  // the queue holds at least (R + DB + 1) SP steps before every round (or every row is done):
  // the prologue takes DB + 1 slots and a round R, so a slot is empty only once every row is done
  auto refill = [&]() {
    while (!done && qh - qt < (R + DB + 1) * SP) {
      const int nun = merge();
      if (nun == 0) done = true;
      qh += nun;
    }
  };
  refill();
#pragma unroll
  for (int s = 0; s < DB + 1; ++s) load_a(s);
#pragma unroll
  for (int s = 0; s < DB; ++s) load_b(s);
  while (vr[0]) {
#pragma unroll
    for (int s = 0; s < R; ++s) {  // a step past the end multiplies nothing (act 0)
      load_a((s + DB + 1) % R);
      load_b((s + DB) % R);
      consume(s);
    }
    asm volatile("" : "+a"(u0), "+a"(u1));  // the accumulators stay in AGPRs through the merge
    refill();
    asm volatile("" : "+a"(u0), "+a"(u1));
  }

  // A tile that met a non-finite B value is left to bsr_small_kernel (the next launch):
  // 0 * inf would reach the rows of block rows without a value in that column. Such a
  // value, multiplied into all 32 rows (by a or by 0), leaves an accumulator inf or NaN,
  // and no finite product does short of overflow (which bsr_small_kernel repeats), so
  // the accumulators tell.
  // the accumulators were last written by MFMAs hipcc may not see through the asm pins:
  // 24 wait states before the first read (MFMA -> VALU read of its result)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(u0), "+a"(u1));
  unsigned mx = 0;
#pragma unroll
  for (int e = 0; e < 32; ++e)
    mx = max(mx, max(__float_as_uint(u0[e]) & 0x7fffffffu, __float_as_uint(u1[e]) & 0x7fffffffu));
  const bool nonfinite = __builtin_amdgcn_ballot_w64(mx >= 0x7f800000u) != 0;
  if (lane == 0) dirty[g * gridDim.y + blockIdx.y] = nonfinite ? 1 : 0;
  if (nonfinite) return;
  const size_t row0 = (size_t)g * 32;
  if constexpr (CROW) {
    const int col = jt + 4 * j;
    if (col >= n) return;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      if (g * G + row / BS >= mb) continue;
      f32x4* p = reinterpret_cast<f32x4*>(C + (row0 + row) * ldc + col);
      f32x4 v = {u0[e], u1[e], u0[16 + e], u1[16 + e]};
      if (beta == 0.f) {
        v *= alpha;
      } else {
        const f32x4 c = *p;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
      }
      *p = v;
    }
  } else {
    constexpr int kTs = 36;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      tile[(4 * j) * kTs + row] = u0[e];
      tile[(4 * j + 1) * kTs + row] = u1[e];
      tile[(4 * j + 2) * kTs + row] = u0[16 + e];
      tile[(4 * j + 3) * kTs + row] = u1[16 + e];
    }
    __syncthreads();
    if (g * G + j / BS < mb) {
      for (int it = 0; it < 64; ++it) {
        const int jl = 2 * it + h;
        if (jt + jl < n) {
          float* p = C + (size_t)(jt + jl) * ldc + row0 + j;
          *p = epi(tile[jl * kTs + j], alpha, beta, p);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Generic VALU kernel: any bs, any storage. Thread = one output element per
// row step; block = (64 columns) x (4 row lanes), grid = (mb, ceil(n/64)).
// Accumulation order: blocks of the block row in order, k = 0..bs-1 inside.
// ---------------------------------------------------------------------------
template <typename TV>
__global__ __launch_bounds__(256) void bsr_generic_kernel(
    int mb, int n, int bs, bool rowdir, const int* __restrict__ rowptr,
    const int* __restrict__ colind, const TV* __restrict__ val, const TV* __restrict__ B, int ldb,
    bool brow, float alpha, float beta, float* __restrict__ C, int ldc, bool crow) {
  const int jj = threadIdx.x & 63;
  const int rl = threadIdx.x >> 6;
  const int br = blockIdx.x;
  const int j = blockIdx.y * 64 + jj;
  if (j >= n) return;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const size_t bs2 = (size_t)bs * bs;
  for (int rr = rl; rr < bs; rr += 4) {
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) {
      const size_t bc = (size_t)colind[k] * bs;
      const TV* ab = val + (size_t)k * bs2;
      for (int c = 0; c < bs; ++c) {
        const float av = (float)(rowdir ? ab[rr * bs + c] : ab[c * bs + rr]);
        const float bv = (float)(brow ? B[(bc + c) * ldb + j] : B[(size_t)j * ldb + bc + c]);
        acc = __builtin_fmaf(av, bv, acc);
      }
    }
    const size_t row = (size_t)br * bs + rr;
    float* p = crow ? C + row * ldc + j : C + (size_t)j * ldc + row;
    *p = epi(acc, alpha, beta, p);
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16, GROUPED item stream (spmm_bsr16_group_analysis_f16 once per
// matrix + spmm_bsrmm_grouped_f16). What bounds the column stream above is the
// B-row gather (40 GB through the texture path per launch on the
// products stand-in, B 34.7 GB of it for 2.5 GB of distinct rows): every
// (block row, nonzero column) pair copies its B row, and neighbouring block
// rows of a reordered graph need mostly the same rows. A workgroup here owns W
// adjacent block rows (one wave each) and streams the UNION of their nonzero
// columns (products stand-in: 0.43 of the pairs at W = 4, 0.29 at W = 8):
//  * an item is 16 union entries (block column J, column c), in (J, c) order;
//    its 16 B rows are copied ONCE into an LDS stage shared by the W waves
//    (8 whole-row copies of 1 KB, split over the waves; the stage layout and
//    the transposed reads are the column stream's FLR ones);
//  * each wave's A fragment of the item (its block row's values of the 16
//    entries, zero where its row stores no such column) was built by the
//    analysis: one 8-B load per lane;
//  * a ring of P stages: per item every wave waits for its own copies (the
//    counted ladder), one s_barrier publishes the stage and retires the slot the
//    next copies overwrite, then 16 transposed reads and 16 MFMAs per wave;
//  * an item's row indices come by scalar loads one item ahead (a vector load
//    would retire behind the copies issued before it and hold the ring to one
//    item in flight), and groups go to the XCDs in chunks of 32 block rows,
//    the column tiles of a group consecutive on one XCD (the later tiles read
//    the A fragments from L2).
// Release form: W = 4, P = 3, three waves per SIMD, one item per barrier:
// products stand-in K = 512 2.44-2.62 ms against 3.77 for the column stream
// (profiles/r04n/, profiles/r04o/).
// Non-finite B: column-granular, as the drop-in stream (round 5). The analysis
// records per (item, wave) which entries the wave's block row holds with a value
// other than +-0; the wave zeroes the other entries' values in its B fragments
// before the MFMAs, so an inf / NaN in a B row reaches only the block rows that
// hold a value in its column (round 4's GROUPED contract let it reach every row
// of the group through the fragments' zeros).
// ---------------------------------------------------------------------------

template <int W, int P, bool CROW, int OCC = 0, int IPB = 1, bool AL = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1)))
void bsr16_f16_grp_kernel(
    int mb, int n, const int* __restrict__ item_ptr, const int* __restrict__ rows,
    const unsigned* __restrict__ wmask, const unsigned* __restrict__ afrag,
    const _Float16* __restrict__ B, int ldb, float alpha, float beta, float* __restrict__ C,
    int ldc, int xm, int ngroups, int ntt) {
  static_assert(W == 2 || W == 4 || W == 8, "waves per group");
  static_assert(P >= 2 && P <= 6, "stages");
  constexpr int COLS = 256, kRowB = 512, kCh = 32, kT = 16, kStage = 16 * kRowB;
  constexpr int kCpw = 8 / W;  // 1-KB copies per wave per item (8 per item)
  constexpr int kSw = 2;       // FLR swizzle: chunk c of row R at 16-B slot (c + 2R) & 31
  // AL (TUNING A/B): the W waves' A fragments of an item come by LDS-DMA beside its B rows
  // (1 KB per copy: two waves' fragments), W / 2 copies per item instead of W 8-B loads
  static_assert(!AL || IPB == 1, "fragments through LDS: one item per barrier");
  constexpr int kSlot = kStage + (AL ? W * 512 : 0);  // bytes per ring slot
  __shared__ __attribute__((aligned(16))) char smem[P * kSlot];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int g = lane >> 4, r16 = lane & 15;
  // neighbouring groups share B rows: chunks of xm groups per XCD keep them in one L2.
  // ntt > 0 (tiles together): a 1-D grid of 8 ceil(ngroups / 8) ntt workgroups in which
  // the ntt column tiles of a group are consecutive on one XCD (dispatch puts workgroup L on
  // XCD L % 8), so the later tiles read the group's A fragments from that L2
  int grp, tile;
  if (ntt > 0) {
    const int L = blockIdx.x, x = L & 7, i = L >> 3;
    const int b = x + 8 * (i / ntt);
    if (b >= ngroups) return;  // the grid's padding (whole workgroup)
    grp = xcd_block_row(b, ngroups, xm);
    tile = i % ntt;
  } else {
    grp = xcd_block_row(blockIdx.x, gridDim.x, xm);
    tile = blockIdx.y;
  }
  const int br = grp * W + w;
  const int jt = tile * COLS;
  const int i0 = item_ptr[grp], i1 = item_ptr[grp + 1];
  const unsigned lds0 = lds_addr(smem);
  const size_t ldb2 = (size_t)ldb * 2;
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 2 * (size_t)jt;

  // this wave's copies: copy cc = w * kCpw + j brings item rows 2 cc (lanes 0-31), 2 cc + 1
  unsigned boffr[kCpw];
#pragma unroll
  for (int j = 0; j < kCpw; ++j) {
    const int R = 2 * (w * kCpw + j) + (lane >> 5);
    boffr[j] = 2u * (unsigned)min(jt + 8 * (((lane & 31) - kSw * R) & (kCh - 1)), n - 8);
  }
  unsigned tra[kT];
  {
    const int R = 4 * g + ((lane >> 2) & 3);
#pragma unroll
    for (int t = 0; t < kT; ++t)
      tra[t] = lds0 + (unsigned)kRowB * R +
               16u * ((2 * t + ((lane & 3) >> 1) + kSw * R) & (kCh - 1)) + 8u * (lane & 1);
  }

  f32x4 acc[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  int nis = 0;  // vector-memory operations issued by this wave
  // row indices of the next IPB items to issue (scalars; rows 2 cc and 2 cc + 1 of copy cc)
  int ra[IPB][kCpw], rb[IPB][kCpw];
  // this wave's held-entry masks (bit e: its block row holds entry e with a value other
  // than +-0): of the next IPB items to issue, and of the items in each ring slot
  unsigned wmn[IPB], wms[P];
  typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
  u32x2a fan[P];  // A fragments in flight (asm-only registers)
  int stamp[P];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    fan[s] = u32x2a{0u, 0u};
    stamp[s] = -64;
    wms[s] = 0u;
  }
#pragma unroll
  for (int i = 0; i < IPB; ++i) {
    wmn[i] = 0u;
#pragma unroll
    for (int j = 0; j < kCpw; ++j) ra[i][j] = rb[i][j] = -1;
  }
  const int ilast = max(i1 - 1, i0);
  // row indices of items it .. it + IPB - 1 (clamped) by scalar loads (lgkmcnt): lane L of
  // copy j needs rows[it][2 (w kCpw + j) + L / 32]. Vector loads retire in issue order
  // behind the copies issued before them, so waiting for a vector row load one item ahead
  // also waited for every copy before it: one item in flight during the MFMAs whatever P
  // was (the grouped stream).
  auto load_rows = [&](int it) {
#pragma unroll
    for (int i = 0; i < IPB; ++i) {
      const int* s2 = rows + (size_t)min(it + i, ilast) * 16 + 2 * w * kCpw;
#pragma unroll
      for (int j = 0; j < kCpw; ++j) {
        ra[i][j] = s2[2 * j];
        rb[i][j] = s2[2 * j + 1];
      }
      wmn[i] = wmask[(size_t)min(it + i, ilast) * W + w];
    }
  };
  // item `it` (rows ra / rb [i]) into stage slot `s`: its copies and A fragment issued
  auto issue = [&](int it, int s, int i) {
    char* const stage = smem + s * kSlot;
    wms[s] = wmn[i];
#pragma unroll
    for (int j = 0; j < kCpw; ++j) {
      const int rw = (lane >> 5) ? rb[i][j] : ra[i][j];
      const char* be = rw >= 0 ? reinterpret_cast<const char*>(B) + (size_t)rw * ldb2 : zrow;
      __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boffr[j]),
                                       (lds_void_t)(stage + 1024 * (w * kCpw + j)), 16, 0, 0);
    }
    if constexpr (AL) {
      // waves 0 .. W / 2 - 1: the fragments of waves 2 w and 2 w + 1 (lanes 0-31 / 32-63)
      if (w < W / 2) {
        const unsigned* fsrc = afrag + ((size_t)min(it, ilast) * W + 2 * w) * 128 + 4 * lane;
        __builtin_amdgcn_global_load_lds((gbl_void_t)fsrc,
                                         (lds_void_t)(stage + kStage + 1024 * w), 16, 0, 0);
        nis += 1;
      }
      nis += kCpw;
    } else {
      const unsigned* fsrc = afrag + ((size_t)min(it, ilast) * W + w) * 128;
      asm volatile("global_load_dwordx2 %0, %1, %2"
                   : "=&v"(fan[s]) : "v"(8u * (unsigned)lane), "s"(fsrc) : "memory");
      nis += kCpw + 1;
    }
    stamp[s] = nis;
  };
  // the 16 transposed reads of slot s and the item's 16 MFMAs
  auto mfma_item = [&](f16x4 fa, auto sc) {
    constexpr int s = decltype(sc)::value;
    f16x4 fb[16];
    asm volatile(
        "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
        "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
        "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
        "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
        "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
        "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
        "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
        "ds_read_b64_tr_b16 %7, %15 offset:%16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]), "=&v"(fb[5]),
          "=&v"(fb[6]), "=&v"(fb[7])
        : "v"(tra[0]), "v"(tra[1]), "v"(tra[2]), "v"(tra[3]), "v"(tra[4]), "v"(tra[5]),
          "v"(tra[6]), "v"(tra[7]), "n"(s * kSlot)
        : "memory");
    asm volatile(
        "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
        "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
        "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
        "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
        "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
        "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
        "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
        "ds_read_b64_tr_b16 %7, %15 offset:%16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(fb[8]), "=&v"(fb[9]), "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]),
          "=&v"(fb[13]), "=&v"(fb[14]), "=&v"(fb[15])
        : "v"(tra[8]), "v"(tra[9]), "v"(tra[10]), "v"(tra[11]), "v"(tra[12]), "v"(tra[13]),
          "v"(tra[14]), "v"(tra[15]), "n"(s * kSlot)
        : "memory");
    // Column-granular non-finite contract: the entries this wave's block row does not
    // hold (its fragment is zero there) have their B values zeroed in the fragment, so
    // an inf / NaN in those B rows meets no 0 * inf. Lane (g, c) holds k = 4 g .. 4 g + 3
    // of the B fragment, as of the A fragment: nibble g of the wave's mask.
    const unsigned wm = wms[s];
    if (wm != 0xffffu) {  // wave-uniform; all 16 held: nothing to clear
      const unsigned nib = (wm >> (4 * g)) & 0xfu;
      const unsigned lo = ((nib & 1u) ? 0xffffu : 0u) | ((nib & 2u) ? 0xffff0000u : 0u);
      const unsigned hi = ((nib & 4u) ? 0xffffu : 0u) | ((nib & 8u) ? 0xffff0000u : 0u);
#pragma unroll
      for (int t = 0; t < kT; ++t) {
        u32x2a v = __builtin_bit_cast(u32x2a, fb[t]);
        v = u32x2a{v[0] & lo, v[1] & hi};
        fb[t] = __builtin_bit_cast(f16x4, v);
      }
    }
#pragma unroll
    for (int t = 0; t < kT; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa, fb[t], acc[t], 0, 0, 0);
  };

  if (i0 < i1) {
    static_assert(P % IPB == 0 && P >= 2 * IPB, "whole barrier groups in the ring");
    // prologue: items i0 .. i0 + P - IPB - 1 in flight, the rows of the next IPB loaded
#pragma unroll
    for (int q = 0; q + IPB < P; q += IPB) {
      load_rows(i0 + q);
#pragma unroll
      for (int i = 0; i < IPB; ++i) issue(i0 + q + i, q + i, i);
    }
    load_rows(i0 + P - IPB);
    // IPB items in slots S IPB .. S IPB + IPB - 1 (static: the fan[] / stage indices)
    auto step = [&](int it, auto sc) {
      constexpr int S = decltype(sc)::value;
      constexpr int s0 = S * IPB;
      // this wave's copies and A fragments of the IPB items landed (in issue order: the
      // last slot's count covers the others); then every wave's, at the barrier
      f16x4 fa[IPB];
      if constexpr (AL) {
        asm volatile(SPMM_VM_LADDER("%0") : : "s"(nis - stamp[s0]) : "scc", "memory");
      } else if constexpr (IPB == 1) {
        u32x2a y;
        asm volatile(SPMM_VM_LADDER("%1") "v_mov_b64 %0, %2"
                     : "=&v"(y) : "s"(nis - stamp[s0]), "v"(fan[s0]) : "scc", "memory");
        fa[0] = __builtin_bit_cast(f16x4, y);
      } else {
        u32x2a y0, y1;
        asm volatile(SPMM_VM_LADDER("%2") "v_mov_b64 %0, %3\n\tv_mov_b64 %1, %4"
                     : "=&v"(y0), "=&v"(y1)
                     : "s"(nis - stamp[s0 + 1]), "v"(fan[s0]), "v"(fan[s0 + 1])
                     : "scc", "memory");
        fa[0] = __builtin_bit_cast(f16x4, y0);
        fa[1] = __builtin_bit_cast(f16x4, y1);
      }
      __builtin_amdgcn_s_barrier();
      if constexpr (AL) {  // this wave's fragment of the item, from the slot's fragment area
        u32x2a y;
        asm volatile("ds_read_b64 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(y)
                     : "v"(lds0 + (unsigned)kStage + 512u * (unsigned)w + 8u * (unsigned)lane),
                       "n"(s0 * kSlot)
                     : "memory");
        fa[0] = __builtin_bit_cast(f16x4, y);
      }
      // the IPB slots before s0 were read by every wave in the previous step: refill them
#pragma unroll
      for (int i = 0; i < IPB; ++i) issue(it + P - IPB + i, (s0 + P - IPB + i) % P, i);
      mfma_item(fa[0], std::integral_constant<int, s0>{});
      // after the first transposed reads: their asm lgkmcnt(0) would also wait for these
      load_rows(it + P);
      if constexpr (IPB == 2) {
        if (it + 1 < i1) mfma_item(fa[1], std::integral_constant<int, s0 + 1>{});
      }
    };
    // whole rounds of P items, then the last < P with no edge back into the loop: a
    // break out of the middle of an unrolled round, merged by the compiler with the
    // latch, would reach the loop head with a slot's A fragment still in flight in a
    // register the head is free to reuse (a path the trip count rules out, but the
    // ISA check, tests/test_isa_waits.py, is path-insensitive and so is the allocator)
    int base = i0;
    for (; base + P <= i1; base += P)
      slots_while(std::make_integer_sequence<int, P / IPB>{}, [&](auto sc) {
        step(base + IPB * decltype(sc)::value, sc);
        return true;
      });
    // uniform over the workgroup: every wave runs the same items
    slots_while(std::make_integer_sequence<int, P / IPB>{}, [&](auto sc) {
      if (base + IPB * decltype(sc)::value >= i1) return false;
      step(base + IPB * decltype(sc)::value, sc);
      return true;
    });
  }
  // nothing in flight past here (the prefetches of clamped items included); the
  // registers those loads fill stay reserved until this wait (uses after it)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < P; ++s) asm volatile("" : : "v"(fan[s]));
  if (br >= mb) return;
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const int j = jt + 16 * t + r16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 32 fp32, GROUPED item stream (spmm_bsr32_group_analysis_f32 once per
// matrix + spmm_bsrmm_grouped_f32; row-major B and C, K tiles of 128). The bs 16
// grouped stream's idea on the fp32 column stream (bsr32_f32_cs2_kernel): a
// workgroup owns W = 2 or 4 adjacent block rows, one wave each, and streams the
// union of their nonzero columns (J, c) in items of 8; an item's 8 B rows (512 B
// at K = 128) are copied once into an LDS stage shared by the W waves. Unlike
// bs 16, where one MFMA takes 16 entries whatever rows hold them, a fp32 MFMA
// here is k = 1 (v_mfma_f32_32x32x1_2b_f32, two per column for 128 outputs),
// so each wave multiplies only the columns its own block row holds: the
// analysis stores a per-(item, wave) mask and the MFMAs of the other columns
// are skipped (wave-uniform branches). A wave's MFMAs are then exactly those of
// the column streams, in the same (J, c) order, so C is bit-identical to
// spmm_bsrmm_ex_f32 / spmm_bsrmm_analysed_f32, and the non-finite contract is
// theirs (column-granular).
//  * per item and wave: its copies (8 / (2 W) of 1 KB: rows 2 cc and 2 cc + 1),
//    one 16-B load of its A fragment (rows j, the item's 8 columns; lane (j, h)
//    columns 4 h .. 4 h + 3, the other four by v_permlane32_swap); row indices
//    and the mask by scalar loads one ring turn ahead (a vector load would
//    retire behind the copies issued before it);
//  * a ring of P stages: counted wait on the wave's own copies and fragment,
//    one s_barrier, the refill of the slot the previous item freed, 8 ds_read_b64
//    of the stage (lane (j, h): columns 4 j + 2 h, + 1 of each row), then per
//    held column two MFMAs.
// Groups go to the XCDs in chunks of xm groups (neighbouring groups share B rows).
// ---------------------------------------------------------------------------
template <int W, int P, int OCC = 0, bool NOMFMA = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1)))
void bsr32_f32_grp_kernel(
    int mb, int n, const int* __restrict__ item_ptr, const int* __restrict__ rows,
    const unsigned* __restrict__ wmask, const float* __restrict__ afrag,
    const float* __restrict__ B, int ldb, float alpha, float beta, float* __restrict__ C, int ldc,
    int xm) {
  static_assert(W == 2 || W == 4, "waves per group");
  static_assert(P >= 2 && P <= 6, "stages");
  constexpr int E = 8, kRowB = 512, kStage = E * kRowB;
  constexpr int kCpw = E / (2 * W);  // 1-KB copies per wave per item
  __shared__ __attribute__((aligned(16))) char smem[P * kStage];
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int grp = xcd_block_row(blockIdx.x, gridDim.x, xm);
  const int br = grp * W + w;
  const int jt = blockIdx.y * 128;
  const int i0 = item_ptr[grp], i1 = item_ptr[grp + 1];
  const unsigned lds0 = lds_addr(smem);
  const size_t ldb4 = (size_t)ldb * 4;
  // copy lanes: 16 B at columns jt + 4 (lane & 31) .. + 3 (n % 4 == 0; clamped in bounds)
  const unsigned boff = 4u * (unsigned)min(jt + 4 * (lane & 31), n - 4);
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 4 * (size_t)jt;
  const unsigned rd = lds0 + 16u * (unsigned)j + 8u * (unsigned)h;  // B reads of the stage

  f32x32 u0, u1;
#pragma unroll
  for (int e = 0; e < 32; ++e) u0[e] = u1[e] = 0.f;

  int nis = 0;  // vector-memory operations issued by this wave
  int ra[kCpw], rb[kCpw];  // row indices of the next item to issue (scalars)
  unsigned msk[P];         // this wave's held columns of the item in each slot (scalars)
  typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
  u32x2a fan[P], fbn[P];  // A fragments in flight, columns 4 h, + 1 / 4 h + 2, + 3 (asm only)
  int stamp[P];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    fan[s] = fbn[s] = u32x2a{0u, 0u};
    stamp[s] = -64;
    msk[s] = 0u;
  }
#pragma unroll
  for (int q = 0; q < kCpw; ++q) ra[q] = rb[q] = -1;
  const int ilast = max(i1 - 1, i0);
  auto load_rows = [&](int it) {
    const int* s2 = rows + (size_t)min(it, ilast) * E + 2 * w * kCpw;
#pragma unroll
    for (int q = 0; q < kCpw; ++q) {
      ra[q] = s2[2 * q];
      rb[q] = s2[2 * q + 1];
    }
  };
  // an item past the group's end holds no columns (its copies are the clamped last item's)
  auto load_mask = [&](int it) -> unsigned {
    return it < i1 ? wmask[(size_t)it * W + w] : 0u;
  };
  auto issue = [&](int it, int s) {
    char* const stage = smem + s * kStage;
#pragma unroll
    for (int q = 0; q < kCpw; ++q) {
      const int rw = h ? rb[q] : ra[q];
      const char* be = rw >= 0 ? reinterpret_cast<const char*>(B) + (size_t)rw * ldb4 : zrow;
      __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boff),
                                       (lds_void_t)(stage + 1024 * (w * kCpw + q)), 16, 0, 0);
    }
    const float* fsrc = afrag + ((size_t)min(it, ilast) * W + w) * 256;
    asm volatile("global_load_dwordx2 %0, %2, %3\n\t"
                 "global_load_dwordx2 %1, %2, %3 offset:8"
                 : "=&v"(fan[s]), "=&v"(fbn[s])
                 : "v"(32u * (unsigned)j + 16u * (unsigned)h), "s"(fsrc)
                 : "memory");
    nis += kCpw + 2;
    stamp[s] = nis;
  };

  if (i0 < i1) {
    load_rows(i0);
#pragma unroll
    for (int q = 0; q + 1 < P; ++q) {
      msk[q] = load_mask(i0 + q);
      issue(i0 + q, q);
      load_rows(i0 + q + 1);
    }
    msk[P - 1] = load_mask(i0 + P - 1);
    auto step = [&](int it, auto sc) {
      constexpr int s = decltype(sc)::value;
      unsigned fa[4];
      {
        u32x2a y0, y1;
        asm volatile(SPMM_VM_LADDER("%2") "v_mov_b64 %0, %3\n\tv_mov_b64 %1, %4"
                     : "=&v"(y0), "=&v"(y1)
                     : "s"(nis - stamp[s]), "v"(fan[s]), "v"(fbn[s])
                     : "scc", "memory");
        fa[0] = y0[0];
        fa[1] = y0[1];
        fa[2] = y1[0];
        fa[3] = y1[1];
      }
      __builtin_amdgcn_s_barrier();
      // slot (s + P - 1) % P was read by every wave in the previous item: refill it
      issue(it + P - 1, (s + P - 1) % P);
      f32x2 fb[E];
      asm volatile(
          "ds_read_b64 %0, %8 offset:%9\n\t"
          "ds_read_b64 %1, %8 offset:%10\n\t"
          "ds_read_b64 %2, %8 offset:%11\n\t"
          "ds_read_b64 %3, %8 offset:%12\n\t"
          "ds_read_b64 %4, %8 offset:%13\n\t"
          "ds_read_b64 %5, %8 offset:%14\n\t"
          "ds_read_b64 %6, %8 offset:%15\n\t"
          "ds_read_b64 %7, %8 offset:%16\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]), "=&v"(fb[5]),
            "=&v"(fb[6]), "=&v"(fb[7])
          : "v"(rd), "n"(s * kStage), "n"(s * kStage + 512), "n"(s * kStage + 1024),
            "n"(s * kStage + 1536), "n"(s * kStage + 2048), "n"(s * kStage + 2560),
            "n"(s * kStage + 3072), "n"(s * kStage + 3584)
          : "memory");
      const unsigned m = msk[s];
      // after the LDS reads: their asm lgkmcnt(0) would also wait for these scalar loads
      load_rows(it + P);
      msk[s] = load_mask(it + P);
      float a[E];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto r = __builtin_amdgcn_permlane32_swap(fa[q], fa[q], false, false);
        a[q] = __uint_as_float(r[0]);
        a[4 + q] = __uint_as_float(r[1]);
      }
      if constexpr (NOMFMA) {  // TUNING diagnostic only (wrong results): the stream without MFMAs
        asm volatile("" : : "v"(a[0]), "v"(a[4]), "v"(fb[0]), "v"(fb[7]), "s"(m));
      } else {
#pragma unroll
        for (int c = 0; c < E; ++c) {
          if (m & (1u << c)) {
            u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(a[c], fb[c][0], u0, 0, 0, 0);
            u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(a[c], fb[c][1], u1, 0, 0, 0);
          }
        }
      }
    };
    int base = i0;
    for (; base + P <= i1; base += P)
      slots_while(std::make_integer_sequence<int, P>{}, [&](auto sc) {
        step(base + decltype(sc)::value, sc);
        return true;
      });
    // uniform over the workgroup: every wave runs the same items
    slots_while(std::make_integer_sequence<int, P>{}, [&](auto sc) {
      if (base + decltype(sc)::value >= i1) return false;
      step(base + decltype(sc)::value, sc);
      return true;
    });
  }
  // nothing in flight past here (the prefetches of clamped items included)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+a"(u0), "+a"(u1) : : "memory");
#pragma unroll
  for (int s = 0; s < P; ++s) asm volatile("" : : "v"(fan[s]), "v"(fbn[s]));
  if (br >= mb) return;
  const int col = jt + 4 * j;
  if (col >= n) return;
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> AGPR read
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    f32x4* p = reinterpret_cast<f32x4*>(C + row * ldc + col);
    f32x4 v;
    asm volatile("v_accvgpr_read_b32 %0, %4\n\t"
                 "v_accvgpr_read_b32 %1, %5\n\t"
                 "v_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3])
                 : "a"(u0[e]), "a"(u1[e]), "a"(u0[16 + e]), "a"(u1[16 + e])
                 : "memory");
    if (beta == 0.f) {
      v *= alpha;
    } else {
      const f32x4 c = *p;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __builtin_fmaf(beta, c[i], alpha * v[i]);
    }
    __builtin_nontemporal_store(v, p);  // C written once (products 2.05 -> 2.00 ms, profiles/r06/ab_ntc.log)
  }
}

// Fallback register-fragment kernels (layouts the copy kernels do not cover):
// bsr32_f32_mfma_kernel / bsr16_*_mfma_kernel variant VAR (launch bounds and
// prefetch form; the best of the round-1 sweep, DESIGN.md §4 "Variant history").
constexpr int kBsr32Default = 40;
constexpr int kBsr16Default = 8;      // fp32 bs 16
constexpr int kBsr16F16Default = 12;  // fp16 bs 16

// Shipped kernels of the ROW-block, row-major-B path, and the alternatives a
// TUNING build (make TUNING=1, -DSPMM_TUNING) lets SPMM_BSR_VARIANT select for
// A/B timing. A release build compiles the override out (variant_override()
// is the constant -1), so no environment setting can change which kernel
// computes a product; the parity subset of each alternative is on record per
// value in profiles/r04_var_tests/ (tools/gpu_var.sh, a TUNING build).
// History of the removed variants: DESIGN.md §4.
//  bs 32 fp32 (bsr32_f32_cs2_kernel: 6 item slots, 3 A slots, 32-bit B-row
//  offsets, cross-block pairs, nt A copies): products stand-in 3.07 ms
//  against 3.15 without nt A (4516, round 2's default), reddit 1.93 / 2.04
//  (profiles/r03_var_sweep.jsonl). 4496: the same without 32-bit offsets,
//  for 32 * ldb * 4 >= 2^31. 4126, not selectable: the full-panel LDS kernel
//  (D = 2, 40 KB, 4 workgroups per CU), the default for blocks known to be
//  dense (the hybrid's BSR part, MFMA-pipe bound: products part 1.71 vs 1.87
//  ms at D = 3) and the kernel of SPMM_BSR_DENSE_BLOCK_PRODUCT. It computes
//  the dense block product (an inf / NaN in a B row only explicit zeros meet
//  reaches C).
constexpr int kBsr32Cs = 4416;
constexpr int kBsr32CsNoNt = 4516;
constexpr int kBsr32CsWideLdb = 4496;
constexpr int kBsr32Dense = 4126;
//  bs 16 fp16, n >= 128 (bsr16_f16_cs_kernel: 2 item stages, 4 A slots, a
//  48-entry pending list, whole-row copies, nt A copies; 19.7 KB of LDS, 8
//  waves per CU), row-major C through an LDS tile (1-KB row stores): products
//  stand-in K = 512 3.79-3.90 ms against 3.91-4.04 storing from the MFMA
//  register layout (profiles/r03_epilogue_ab.txt); 6104 is the same without nt A (4.03 against 3.88
//  before the staged epilogue). Below 128 columns, and 4725: the column-masked
//  block kernel (bsr16_cm_kernel, at least 8 waves per SIMD).
constexpr int kBsr16F16Cs = 6404;
constexpr int kBsr16F16CsNoNt = 6104;
constexpr int kBsr16F16Cm = 4725;
//  bs 16 fp32: the column-masked block kernel (products stand-in K = 512
//  16.6 ms against 18.5 for the full-panel kernel).

#ifdef SPMM_TUNING
// SPMM_SMALL_GRP=0: bs 2 / 4 / 8 on bsr_small_kernel instead of the grouped MFMA
// stream, for A/B timing
bool small_grp_enabled() {
  static const bool on = [] {
    const char* e = getenv("SPMM_SMALL_GRP");
    return !e || atoi(e) != 0;
  }();
  return on;
}
int variant_override() {
  static const int var = [] {
    const char* e = getenv("SPMM_BSR_VARIANT");
    return e ? atoi(e) : -1;
  }();
  return var;
}
// SPMM_BSR_ORDER=1 / 2 / 3 (below): scheduling A/B of the column streams
int order_override() {
  static const int force = [] {
    const char* e = getenv("SPMM_BSR_ORDER");
    return e ? atoi(e) : 0;
  }();
  return force;
}
#else
constexpr bool small_grp_enabled() { return true; }
constexpr int variant_override() { return -1; }
constexpr int order_override() { return 0; }
#endif
#define SPMM_COMMA ,

// Block-row order for the column-stream kernels: longest first when the grid
// is at most kLptRounds waves per resident slot deep (a few long rows would
// otherwise start last and run alone), else nullptr (the kernels' XCD-chunked
// order, which keeps neighbouring block rows in one L2). In a TUNING build
// SPMM_BSR_ORDER=1 forces longest first, 2 the XCD order. One launch of
// block_row_order_kernel into the handle's order buffer, in stream order.
constexpr int kLptRounds = 8;

// Segments for the bs = 32 column stream with row-major C (seg_build_kernel):
// on a shallow grid (the block_row_order rule), when the longest row holds
// more than twice the mean load per wave slot (2 nnzb / slots blocks), rows
// longer than L = max(64, nnzb / (2 * slots)) blocks are split. Fills the segment and
// split-row lists (order buffer) and the partial tiles (workspace); *segs stays
// nullptr on a deep grid or with SPMM_BSR_ORDER=2 / 3 (3: longest first, no
// splitting).
spmm_status_t cs2_segments(spmm_context* ctx, int mb, int nnzb, int ntiles, const int* rowptr,
                           const int4** segs, const int4** splits, float** part, int* nseg,
                           int* nsplit) {
  const int force = order_override();
  *segs = nullptr;
  *splits = nullptr;
  *part = nullptr;
  const long slots = 12L * ctx->num_cus;
  if (force == 2 || force == 3 || (force != 1 && (long)mb * ntiles > kLptRounds * slots) || nnzb <= 0)
    return SPMM_STATUS_SUCCESS;
  const int L = (int)std::max<long>(64, ((long)nnzb + 2 * slots - 1) / (2 * slots));
  const int split_cap = nnzb / L + 1;
  const int seg_cap = mb + split_cap;
  const size_t parts_cap = 2 * (size_t)split_cap;
  if (spmm_status_t st = spmm::ensure_order_buffer(ctx, 4 * ((size_t)seg_cap + split_cap))) return st;
  if (spmm_status_t st = spmm::ensure_scratch(ctx, parts_cap * ntiles * 32 * 128 * sizeof(float)))
    return st;
  int4* sg = reinterpret_cast<int4*>(ctx->order);
  int4* sp = sg + seg_cap;
  const int split_if = (int)std::min<long>(0x7fffffff, 2 * ((long)nnzb + slots - 1) / slots);
  hipLaunchKernelGGL(seg_build_kernel, dim3(1), dim3(1024), 0, ctx->stream, mb, rowptr, L, split_if,
                     seg_cap, split_cap, (int)parts_cap, sg, sp);
  *segs = sg;
  *splits = sp;
  *part = reinterpret_cast<float*>(ctx->scratch);
  *nseg = seg_cap;
  *nsplit = split_cap;
  return SPMM_STATUS_SUCCESS;
}
spmm_status_t block_row_order(spmm_context* ctx, int mb, int ntiles, const int* rowptr,
                              const int** order, long slots_per_cu = 12, const int* crp = nullptr,
                              int m = 0, int sub = 0) {
  const int force = order_override();
  *order = nullptr;
  const long waves = (long)mb * ntiles, slots = slots_per_cu * ctx->num_cus;
  if (force == 2 || (force != 1 && force != 3 && waves > kLptRounds * slots))
    return SPMM_STATUS_SUCCESS;
  if (spmm_status_t st = spmm::ensure_order_buffer(ctx, mb)) return st;
  hipLaunchKernelGGL(block_row_order_kernel, dim3(1), dim3(1024), 0, ctx->stream, mb, rowptr,
                     crp, m, sub, ctx->order);
  *order = ctx->order;
  return SPMM_STATUS_SUCCESS;
}

#define SPMM_BSR_DISPATCH(KERNEL, TA, GRID, BLOCK, STREAM, ROWD, BR, CR, ...)                 \
  do {                                                                                    \
    if (ROWD) {                                                                           \
      if (BR) {                                                                           \
        if (CR) hipLaunchKernelGGL((KERNEL<true, true, true TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);   \
        else hipLaunchKernelGGL((KERNEL<true, true, false TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);     \
      } else {                                                                            \
        if (CR) hipLaunchKernelGGL((KERNEL<true, false, true TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else hipLaunchKernelGGL((KERNEL<true, false, false TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);    \
      }                                                                                   \
    } else {                                                                              \
      if (BR) {                                                                           \
        if (CR) hipLaunchKernelGGL((KERNEL<false, true, true TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else hipLaunchKernelGGL((KERNEL<false, true, false TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);    \
      } else {                                                                            \
        if (CR) hipLaunchKernelGGL((KERNEL<false, false, true TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__); \
        else hipLaunchKernelGGL((KERNEL<false, false, false TA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);   \
      }                                                                                   \
    }                                                                                     \
  } while (0)

bool aligned(const void* p, int bytes) { return reinterpret_cast<uintptr_t>(p) % bytes == 0; }

}  // namespace

namespace spmm {

spmm_status_t launch_bsr32_analysis(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                    const float* val, unsigned* masks, float* val_col) {
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  hipLaunchKernelGGL(bsr32_analysis_kernel, dim3((nnzb + 3) / 4), dim3(256), 0, ctx->stream, nnzb,
                     dir == SPMM_DIRECTION_ROW ? 1 : 0, val, masks, val_col);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsr16_analysis(spmm_context* ctx, spmm_direction_t dir, int nnzb,
                                    const uint16_t* val, unsigned* masks, uint16_t* val_col) {
  if (nnzb == 0) return SPMM_STATUS_SUCCESS;
  const long long per_block = 4 * kAna16Bpw;  // 4 waves, kAna16Bpw blocks each
  hipLaunchKernelGGL(bsr16_analysis_kernel, dim3((unsigned)((nnzb + per_block - 1) / per_block)),
                     dim3(256), 0, ctx->stream, nnzb, dir == SPMM_DIRECTION_ROW ? 1 : 0, val,
                     masks, val_col);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsrmm_f32(spmm_context* ctx, spmm_direction_t dir, int mb, int kb, int n,
                               int nnzb, int bs, float alpha, const int* rowptr,
                               const int* colind, const float* val, const float* B, int ldb,
                               spmm_order_t orderB, float beta, float* C, int ldc,
                               spmm_order_t orderC, bool dense_blocks, const unsigned* masks) {
  (void)kb;
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const bool rowd = dir == SPMM_DIRECTION_ROW;
  const bool brow = orderB == SPMM_ORDER_ROW;
  const bool crow = orderC == SPMM_ORDER_ROW;
  const bool vec_ok = aligned(val, 16) && (brow || (aligned(B, 16) && ldb % 4 == 0));
  const int slot = timing_begin(ctx);
  const int var = variant_override();
  // SPMM_BSR_DENSE_BLOCK_PRODUCT: cusparseSbsrmm's dense-block semantics, the full-panel
  // kernels only (no column masks); the split-bf16 option stays the hybrid's own
  const bool hybrid_part = dense_blocks;
  const bool dense_sem = (ctx->bsr_flags & SPMM_BSR_DENSE_BLOCK_PRODUCT) != 0;
  if (dense_sem) {
    dense_blocks = true;
    masks = nullptr;
  }
  // the column stream stores row-major C as 16-B row pieces (and its segment fix-up too):
  // C and ldc must keep them aligned, else the fragment kernel's scalar stores serve
  const bool c16 = !crow || (aligned(C, 16) && ldc % 4 == 0);
  // the analysed column stream: COLUMN blocks with their column masks
  const bool msk = masks && bs == 32 && !rowd && !dense_blocks && c16;
  if (bs == 32 && (rowd || msk) && brow && n >= 4 && n % 4 == 0 && ldb % 4 == 0 &&
      aligned(val, 16) && aligned(B, 16) && (dense_blocks || c16)) {
    const dim3 grid(mb, (n + 127) / 128);
    const bool narrow = (size_t)ldb * 128 < (1u << 31);  // 32-row panels addressable in 31 bits
    int lv = dense_blocks ? kBsr32Dense : kBsr32Cs;
    // (a tuning override never replaces the dense-block kernel: the hybrid's
    // column-major form stages B in the handle scratch the column stream's
    // segments would reuse)
    if (!dense_blocks && (var == kBsr32CsNoNt || var == kBsr32CsWideLdb || var == kBsr32Cs))
      lv = var;
    if (!narrow && (lv == kBsr32Cs || lv == kBsr32CsNoNt)) lv = kBsr32CsWideLdb;
    if (lv == kBsr32Dense) {
      // split-bf16 (opt-in, SPMM_HYBRID_SPLIT_BF16): wave-pair split-K for row-major C
      // (products hybrid 1.86-1.87 vs 1.89 ms fused, reddit 0.80 vs 0.83,
      // profiles/r01_hybrid_split.jsonl), one k range per wave for column-major C
      const bool split = hybrid_part && (ctx->hybrid_flags & SPMM_HYBRID_SPLIT_BF16);
      if (split && crow)
        hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, false, 24, true, true>), grid,
                           dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha,
                           beta, C, ldc, nullptr, nullptr, nullptr, 0, nullptr);
      else if (split)
        hipLaunchKernelGGL((bsr32_f32_lds_kernel<false, 2, 32, false, 24, true>), grid,
                           dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha,
                           beta, C, ldc, nullptr, nullptr, nullptr, 0, nullptr);
      else if (crow)
        hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32>), grid, dim3(256), 0, ctx->stream,
                           mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, nullptr,
                           nullptr, nullptr, 0, nullptr);
      else
        hipLaunchKernelGGL((bsr32_f32_lds_kernel<false, 2, 32>), grid, dim3(256), 0, ctx->stream,
                           mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, nullptr,
                           nullptr, nullptr, 0, nullptr);
    } else {
      // the column stream: segments of outlier rows (row-major C, shallow grids) or the
      // longest-first order (shallow grids), else the XCD-chunked order
      const int* ord = nullptr;
      const int4 *sg = nullptr, *spl = nullptr;
      float* pt = nullptr;
      int nsg = 0, nspl = 0;
      spmm_status_t st = SPMM_STATUS_SUCCESS;
      if (crow) st = cs2_segments(ctx, mb, nnzb, grid.y, rowptr, &sg, &spl, &pt, &nsg, &nspl);
      if (st == SPMM_STATUS_SUCCESS && !sg) st = block_row_order(ctx, mb, grid.y, rowptr, &ord);
      if (st != SPMM_STATUS_SUCCESS) {
        timing_end(ctx, slot);
        return st;
      }
      const dim3 g2(sg ? nsg : mb, grid.y);
      // n <= 64: the 64-column tile (C64; grid.y is 1 either way, so the segments'
      // partial layout is the same)
      const bool c64 = n <= 64;
      // the panel stream (same bits) when the probe finds the blocks dense: both kernels go
      // out, the probe's sums choose on the device (no host round trip, graph-capturable)
      unsigned long long* pstat = nullptr;
      if (!msk && !sg && lv == kBsr32Cs && nnzb >= kPanelMinBlocks) {
        if (spmm_status_t st2 = spmm::ensure_scratch(ctx, 2 * sizeof(unsigned long long))) {
          timing_end(ctx, slot);
          return st2;
        }
        pstat = static_cast<unsigned long long*>(ctx->scratch);
        if (hipError_t e = hipMemsetAsync(pstat, 0, 2 * sizeof(*pstat), ctx->stream)) {
          timing_end(ctx, slot);
          return from_hip(e);
        }
        const int ns = std::min(nnzb, kPanelSamples);
        hipLaunchKernelGGL(panel_probe_kernel, dim3((ns + 4 * kPanelPerWave - 1) / (4 * kPanelPerWave)),
                           dim3(256), 0, ctx->stream, (long long)nnzb, ns, 0, val, pstat);
      }
#define CS2_ONE(C64_, O32_, PK_, ANT_)                                                           \
  do {                                                                                           \
    if (crow)                                                                                    \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<true, 32, 6, 3, O32_, PK_, ANT_, false, false,    \
                                               C64_>),                                           \
                         g2, dim3(64), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,       \
                         alpha, beta, C, ldc, ord, sg, pt, masks, pstat);                        \
    else                                                                                         \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<false, 32, 6, 3, O32_, PK_, ANT_, false, false,   \
                                               C64_>),                                           \
                         g2, dim3(64), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,       \
                         alpha, beta, C, ldc, ord, nullptr, nullptr, masks, pstat);              \
  } while (0)
#define CS2_LAUNCH(O32_, PK_, ANT_)                                                              \
  do {                                                                                           \
    if (c64) CS2_ONE(true, O32_, PK_, ANT_);                                                     \
    else CS2_ONE(false, O32_, PK_, ANT_);                                                        \
  } while (0)
#define MSK_ONE(C64_, O32_)                                                                      \
  do {                                                                                           \
    if (crow)                                                                                    \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<true, 32, 6, 3, O32_, true, true, true, false,    \
                                               C64_>),                                           \
                         g2, dim3(64), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,       \
                         alpha, beta, C, ldc, ord, sg, pt, masks);                               \
    else                                                                                         \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<false, 32, 6, 3, O32_, true, true, true, false,   \
                                               C64_>),                                           \
                         g2, dim3(64), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,       \
                         alpha, beta, C, ldc, ord, nullptr, nullptr, masks);                     \
  } while (0)
#define MSK_LAUNCH(O32_)                                                                         \
  do {                                                                                           \
    if (c64) MSK_ONE(true, O32_);                                                                \
    else MSK_ONE(false, O32_);                                                                   \
  } while (0)
      // (4, 8 or 10 items in flight: 2.11-2.15 / 2.11-2.12 / 2.43 ms against 2.11 at 6 on
      // the products stand-in, profiles/r03_analysed_sweep.txt)
      if (msk && narrow) MSK_LAUNCH(true);
      else if (msk) MSK_LAUNCH(false);
#undef MSK_LAUNCH
#undef MSK_ONE
      else if (lv == kBsr32Cs) CS2_LAUNCH(true, true, true);
      else if (lv == kBsr32CsNoNt) CS2_LAUNCH(true, true, false);
      else CS2_LAUNCH(false, true, true);  // kBsr32CsWideLdb
#undef CS2_LAUNCH
#undef CS2_ONE
      if (pstat) {
        if (crow && c64)
          hipLaunchKernelGGL((bsr32_f32_panel_kernel<true, true, SPMM_PANEL_D64>), g2, dim3(64), 0, ctx->stream,
                             mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, ord, pstat);
        else if (crow)
          hipLaunchKernelGGL((bsr32_f32_panel_kernel<true, false, SPMM_PANEL_D128>), g2, dim3(64), 0,
                             ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,
                             ord, pstat);
        else if (c64)
          hipLaunchKernelGGL((bsr32_f32_panel_kernel<false, true, SPMM_PANEL_D64>), g2, dim3(64), 0,
                             ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,
                             ord, pstat);
        else
          hipLaunchKernelGGL((bsr32_f32_panel_kernel<false, false, SPMM_PANEL_D128>), g2, dim3(64), 0,
                             ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,
                             ord, pstat);
      }
      if (spl)
        hipLaunchKernelGGL(seg_fixup_kernel, dim3(nspl, grid.y), dim3(256), 0, ctx->stream, n,
                           spl, pt, alpha, beta, C, ldc);
    }
  } else if (bs == 64 && rowd && brow && n >= 4 && n % 4 == 0 && ldb % 4 == 0 &&
             aligned(val, 16) && aligned(B, 16) && c16 && !dense_sem) {
    // bs 64: the bs 32 column stream on the four 32 x 32 sub-blocks of each block
    // (SUB), one wave per 32-row half of a block row and 128 columns
    const int mb2 = 2 * mb;
    const dim3 g2(mb2, (n + 127) / 128);
    const bool narrow = (size_t)ldb * 128 < (1u << 31);
    const int* ord = nullptr;
    if (const spmm_status_t st = block_row_order(ctx, mb2, g2.y, rowptr, &ord, 12, nullptr, 0, 1)) {
      timing_end(ctx, slot);
      return st;
    }
    // the panel stream over the sub-blocks when the probe finds them dense (same bits)
    unsigned long long* pstat = nullptr;
    if (narrow && 4LL * nnzb >= kPanelMinBlocks) {
      if (spmm_status_t st2 = spmm::ensure_scratch(ctx, 2 * sizeof(unsigned long long))) {
        timing_end(ctx, slot);
        return st2;
      }
      pstat = static_cast<unsigned long long*>(ctx->scratch);
      if (hipError_t e = hipMemsetAsync(pstat, 0, 2 * sizeof(*pstat), ctx->stream)) {
        timing_end(ctx, slot);
        return from_hip(e);
      }
      const long long nsub = 4LL * nnzb;
      const int ns = (int)std::min<long long>(nsub, kPanelSamples);
      hipLaunchKernelGGL(panel_probe_kernel, dim3((ns + 4 * kPanelPerWave - 1) / (4 * kPanelPerWave)),
                         dim3(256), 0, ctx->stream, nsub, ns, 1, val, pstat);
    }
#define SUB_ONE(CR_, O32_, C64_)                                                                 \
  hipLaunchKernelGGL((bsr32_f32_cs2_kernel<CR_, 32, 6, 3, O32_, true, true, false, true, C64_>),  \
                     g2, dim3(64), 0, ctx->stream, mb2, n, rowptr, colind, val, B, ldb, alpha,   \
                     beta, C, ldc, ord, nullptr, nullptr, nullptr, pstat)
#define SUB_LAUNCH(CR_, O32_)                                                                    \
  do {                                                                                           \
    if (n <= 64) SUB_ONE(CR_, O32_, true);  /* the 64-column tile */                             \
    else SUB_ONE(CR_, O32_, false);                                                              \
  } while (0)
    if (crow) {
      if (narrow) SUB_LAUNCH(true, true); else SUB_LAUNCH(true, false);
    } else {
      if (narrow) SUB_LAUNCH(false, true); else SUB_LAUNCH(false, false);
    }
#undef SUB_LAUNCH
#undef SUB_ONE
    if (pstat) {
#define PSUB(CR_, C64_, D_)                                                                       \
  hipLaunchKernelGGL((bsr32_f32_panel_kernel<CR_, C64_, D_, true>), g2, dim3(64), 0, ctx->stream, \
                     mb2, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, ord, pstat)
      if (crow && n <= 64) PSUB(true, true, SPMM_PANEL_D64);
      else if (crow) PSUB(true, false, SPMM_PANEL_D128);
      else if (n <= 64) PSUB(false, true, SPMM_PANEL_D64);
      else PSUB(false, false, SPMM_PANEL_D128);
#undef PSUB
    }
  } else if (bs == 32 && vec_ok) {
    const int waves = n <= 32 ? 1 : (n <= 64 ? 2 : 4);
    dim3 grid(mb, (n + 32 * waves - 1) / (32 * waves));
    SPMM_BSR_DISPATCH(bsr32_f32_mfma_kernel, SPMM_COMMA kBsr32Default, grid, dim3(64 * waves),
                      ctx->stream, rowd, brow, crow, mb, n, rowptr, colind, val, B, ldb, alpha,
                      beta, C, ldc);
  } else if (bs == 16 && rowd && brow && n >= 4 && n % 4 == 0 && ldb % 4 == 0 &&
             aligned(val, 16) && aligned(B, 16) && !dense_sem) {
    // output columns per workgroup: 256, or the narrower tile a small n fills (at n = 64
    // a 256-column tile left 3 of its 4 waves idle: reference sweep, profiles/r05_sweep/)
    const int cols = n <= 64 ? 64 : (n <= 128 ? 128 : 256);
    const dim3 grid(mb, (n + cols - 1) / cols);
#define CM16_LAUNCH(CR_, COLS_)                                                                   \
  hipLaunchKernelGGL((bsr16_cm_kernel<float, CR_, 2, 5, 1, COLS_>), grid, dim3(256), 0,           \
                     ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc)
    if (cols == 64) {
      if (crow) CM16_LAUNCH(true, 64); else CM16_LAUNCH(false, 64);
    } else if (cols == 128) {
      if (crow) CM16_LAUNCH(true, 128); else CM16_LAUNCH(false, 128);
    } else {
      if (crow) CM16_LAUNCH(true, 256); else CM16_LAUNCH(false, 256);
    }
#undef CM16_LAUNCH
  } else if (bs == 16 && vec_ok) {
    const int waves = n <= 64 ? 1 : (n <= 128 ? 2 : 4);
    dim3 grid(mb, (n + 64 * waves - 1) / (64 * waves));
    SPMM_BSR_DISPATCH(bsr16_f32_mfma_kernel, SPMM_COMMA kBsr16Default, grid, dim3(64 * waves),
                      ctx->stream, rowd, brow, crow, mb, n, rowptr, colind, val, B, ldb, alpha,
                      beta, C, ldc);
  } else if ((bs == 2 || bs == 4 || bs == 8) && brow && !dense_sem && nnzb > 0 && n >= 4 &&
             n % 4 == 0 && ldb % 2 == 0 && aligned(B, 8) && aligned(val, 16) &&
             (!crow || (ldc % 4 == 0 && aligned(C, 16))) && kb < (1 << 26) &&
             (size_t)ldb * bs * 4 < (1u << 31) && (size_t)(32 / bs) * kb * bs * bs * 4 < (1u << 31) &&
             (nnzb >= (1 << 20) || (ctx->bsr_flags & SPMM_BSR_SMALL_GROUPED)) &&
             small_grp_enabled()) {
    // (from 2^20 blocks: its fixed cost, the probe and the order, about 40 us, made the
    // reference sweep's small cells up to 2x slower; SPMM_BSR_SMALL_GROUPED forces it)
    // the grouped MFMA stream: 32 / bs block rows per wave share each B row of their union
    const int ngroups = (mb + 32 / bs - 1) / (32 / bs);
    const dim3 grid(ngroups, (n + 127) / 128);
    if (spmm_status_t st = ensure_scratch(ctx, (size_t)ngroups * grid.y * sizeof(int) + 256)) {
      timing_end(ctx, slot);
      return st;
    }
    // the probe's integer sums
    unsigned long long* stat = static_cast<unsigned long long*>(ctx->scratch);
    int* dirty = reinterpret_cast<int*>(static_cast<char*>(ctx->scratch) + 256);
    constexpr int xm = SPMM_SGRP_XM;  // groups per XCD chunk
    // a shallow grid (a few waves per resident slot): groups longest first (reddit bs 8
    // 1.50 -> 1.37 ms: 2.4 waves per slot, group loads up to 2.7x the mean), else the
    // XCD-chunked order
    const int* ord = nullptr;
    dim3 lgrid = grid;
    {
      const long slots = 12L * ctx->num_cus;
      if (SPMM_SGRP_LPT && (long)ngroups * grid.y <= kLptRounds * slots) {
        // chunks of xm groups, longest first (block_row_order_kernel keyed by a chunk's blocks)
        // (chunks of xm groups ranked together, XCD chunks kept: 1.41-1.43 ms on reddit bs 8
        // against 1.37 for single groups, the same box; profiles/r05b/small_grp/)
        const int cx = SPMM_SGRP_LPT == 2 ? xm : 1;
        const int nch = (ngroups + cx - 1) / cx;
        if (spmm_status_t st = spmm::ensure_order_buffer(ctx, nch)) {
          timing_end(ctx, slot);
          return st;
        }
        const double mean = (double)nnzb / nch;
        int gshift = 0;
        while ((4.0 * mean) / (1 << gshift) > 1023.0) ++gshift;
        hipLaunchKernelGGL(block_row_order_kernel, dim3(1), dim3(1024), 0, ctx->stream, nch,
                           rowptr, nullptr, mb, 0, ctx->order, 32 / bs * cx, gshift);
        ord = ctx->order;
        lgrid.x = nch * cx;
      }
    }
#define SGRP_ONE(BS_, RD_, CR_)                                                                  \
  hipLaunchKernelGGL((bsr_small_grp_kernel<BS_, RD_, CR_>), lgrid, dim3(64), 0, ctx->stream, mb, \
                     n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, SPMM_SGRP_LPT != 2 && ord ? 1 : xm, dirty, ord, nnzb, \
                     stat)
#define SGRP_LAUNCH(BS_)                                                                         \
  do {                                                                                           \
    if (rowd && crow) SGRP_ONE(BS_, true, true);                                                 \
    else if (rowd) SGRP_ONE(BS_, true, false);                                                   \
    else if (crow) SGRP_ONE(BS_, false, true);                                                   \
    else SGRP_ONE(BS_, false, false);                                                            \
  } while (0)
    ctx->small_path = 1;  // the probe's sums decide (spmm_bsr_small_path)
    ctx->small_path_bs = bs;
    // the choice per matrix first (small_grp_probe_kernel), then the stream
    if (hipError_t e = hipMemsetAsync(stat, 0, 2 * sizeof(*stat), ctx->stream)) {
      timing_end(ctx, slot);
      return from_hip(e);
    }
    const dim3 pgrid(std::min(ngroups, 1024));
    if (bs == 8)
      hipLaunchKernelGGL(small_grp_probe_kernel<8>, pgrid, dim3(64), 0, ctx->stream, mb, ngroups,
                         rowptr, colind, stat);
    else if (bs == 4)
      hipLaunchKernelGGL(small_grp_probe_kernel<4>, pgrid, dim3(64), 0, ctx->stream, mb, ngroups,
                         rowptr, colind, stat);
    else
      hipLaunchKernelGGL(small_grp_probe_kernel<2>, pgrid, dim3(64), 0, ctx->stream, mb, ngroups,
                         rowptr, colind, stat);
    if (bs == 8) SGRP_LAUNCH(8);
    else if (bs == 4) SGRP_LAUNCH(4);
    else SGRP_LAUNCH(2);
#undef SGRP_LAUNCH
#undef SGRP_ONE
    // the tiles it flagged (a non-finite B value met): bsr_small_kernel recomputes them
    const bool v2 = n > 64;  // n % 4 == 0, ldb % 2 == 0 and B 8-B aligned above
    const dim3 fgrid((mb + 3) / 4, (n + (v2 ? 127 : 63)) / (v2 ? 128 : 64));
#define SFIX_ONE(BS_, V_, RD_, CR_)                                                              \
  hipLaunchKernelGGL((bsr_small_kernel<BS_, V_, RD_, CR_>), fgrid, dim3(256), 0, ctx->stream, mb, \
                     n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, 8, dirty, (int)grid.y)
#define SFIX_LAUNCH(BS_, V_)                                                                     \
  do {                                                                                           \
    if (rowd && crow) SFIX_ONE(BS_, V_, true, true);                                             \
    else if (rowd) SFIX_ONE(BS_, V_, true, false);                                               \
    else if (crow) SFIX_ONE(BS_, V_, false, true);                                               \
    else SFIX_ONE(BS_, V_, false, false);                                                        \
  } while (0)
    if (bs == 8) {
      if (v2) SFIX_LAUNCH(8, 2); else SFIX_LAUNCH(8, 1);
    } else if (bs == 4) {
      if (v2) SFIX_LAUNCH(4, 2); else SFIX_LAUNCH(4, 1);
    } else {
      if (v2) SFIX_LAUNCH(2, 2); else SFIX_LAUNCH(2, 1);
    }
#undef SFIX_LAUNCH
#undef SFIX_ONE
  } else if ((bs == 2 || bs == 4 || bs == 8) && brow && !dense_sem) {
    ctx->small_path = 0;
    // the lane-group VALU kernel: 2 floats per lane when B allows 8-B gathers
    const bool v2 = n > 64 && n % 2 == 0 && ldb % 2 == 0 && aligned(B, 8);
    const dim3 grid((mb + 3) / 4, (n + (v2 ? 127 : 63)) / (v2 ? 128 : 64));
    // XCD chunks of 8 workgroups (32 block rows; TUNING builds: SPMM_SMALL_XM)
#ifdef SPMM_TUNING
    static const int xm = [] {
      const char* e = getenv("SPMM_SMALL_XM");
      return e ? atoi(e) : 8;
    }();
#else
    constexpr int xm = 8;
#endif
#define SMALL_ONE(BS_, V_, RD_, CR_)                                                             \
  hipLaunchKernelGGL((bsr_small_kernel<BS_, V_, RD_, CR_>), grid, dim3(256), 0, ctx->stream, mb, \
                     n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, xm)
#define SMALL_LAUNCH(BS_, V_)                                                                    \
  do {                                                                                           \
    if (rowd && crow) SMALL_ONE(BS_, V_, true, true);                                            \
    else if (rowd) SMALL_ONE(BS_, V_, true, false);                                              \
    else if (crow) SMALL_ONE(BS_, V_, false, true);                                              \
    else SMALL_ONE(BS_, V_, false, false);                                                       \
  } while (0)
    if (bs == 8) {
      if (v2) SMALL_LAUNCH(8, 2); else SMALL_LAUNCH(8, 1);
    } else if (bs == 4) {
      if (v2) SMALL_LAUNCH(4, 2); else SMALL_LAUNCH(4, 1);
    } else {
      if (v2) SMALL_LAUNCH(2, 2); else SMALL_LAUNCH(2, 1);
    }
#undef SMALL_LAUNCH
#undef SMALL_ONE
  } else {
    dim3 grid(mb, (n + 63) / 64);
    hipLaunchKernelGGL(bsr_generic_kernel<float>, grid, dim3(256), 0, ctx->stream, mb, n, bs,
                       rowd, rowptr, colind, val, B, ldb, brow, alpha, beta, C, ldc, crow);
  }
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

bool hybrid32_fusable(int n, int ldb, int ldc, const float* bval, const float* B, const float* C) {
  return n >= 4 && n % 4 == 0 && ldb % 4 == 0 && ldc % 2 == 0 && aligned(bval, 16) &&
         aligned(B, 16) && aligned(C, 8);
}

spmm_status_t launch_hybrid32_fused(spmm_context* ctx, int m, int n, float alpha,
                                    const int* crp, const int* cci, const float* cv,
                                    const int* brp, const int* bci, const float* bval,
                                    const float* B, int ldb, float beta, float* C, int ldc) {
  const int mb = (m + 31) / 32;
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const int slot = timing_begin(ctx);
  const dim3 grid(mb, (n + 127) / 128);
  // longest first (blocks and remainder entries) when the grid is a few
  // workgroups per slot deep (4 workgroups per CU)
  const int* ord = nullptr;
  if (const spmm_status_t st = block_row_order(ctx, mb, grid.y, brp, &ord, 4, crp, m)) {
    timing_end(ctx, slot);
    return st;
  }
  if (ctx->hybrid_flags & SPMM_HYBRID_SPLIT_BF16)  // wave-pair split-K, split-bf16 products
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, true, 24, true, true>), grid, dim3(256), 0,
                       ctx->stream, mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else  // D = 2 and 24 remainder gathers in flight (73 VGPRs): 4 workgroups per CU.
        // Products stand-in 2.09 ms vs 2.42 with 32 in flight and 2.81 with D = 3.
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, true, 24>), grid, dim3(256), 0,
                       ctx->stream, mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsrmm_f16(spmm_context* ctx, spmm_direction_t dir, int mb, int kb, int n,
                               int nnzb, int bs, float alpha, const int* rowptr,
                               const int* colind, const uint16_t* val16, const uint16_t* B16,
                               int ldb, spmm_order_t orderB, float beta, float* C, int ldc,
                               spmm_order_t orderC, const unsigned* masks) {
  (void)kb;
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const _Float16* val = reinterpret_cast<const _Float16*>(val16);
  const _Float16* B = reinterpret_cast<const _Float16*>(B16);
  const bool rowd = dir == SPMM_DIRECTION_ROW;
  const bool brow = orderB == SPMM_ORDER_ROW;
  const bool crow = orderC == SPMM_ORDER_ROW;
  const bool vec_ok = aligned(val, 16) && (brow || (aligned(B, 16) && ldb % 8 == 0));
  const int slot = timing_begin(ctx);
  const int var = variant_override();
  // SPMM_BSR_DENSE_BLOCK_PRODUCT: the register-fragment kernel (dense blocks, no masks)
  const bool dense_sem = (ctx->bsr_flags & SPMM_BSR_DENSE_BLOCK_PRODUCT) != 0;
  // the analysed column stream: COLUMN blocks with their column masks, n >= 128
  const bool msk = masks && bs == 16 && !rowd && n >= 128 && !dense_sem;
  if (bs == 16 && (rowd || msk) && brow && n >= 8 && n % 8 == 0 && ldb % 8 == 0 &&
      aligned(val, 16) && aligned(B, 16) && !dense_sem) {
    int lv = n >= 128 ? kBsr16F16Cs : kBsr16F16Cm;
    if (var == kBsr16F16Cm ||
        (n >= 128 && (var == kBsr16F16Cs || var == kBsr16F16CsNoNt)))
      lv = var;
    if (msk) lv = kBsr16F16Cs;  // COLUMN blocks: only the analysed stream reads them here
    if (lv == kBsr16F16Cm) {
      const dim3 grid(mb, (n + 255) / 256);
      if (crow)
        hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, true, 2, 5, 8>), grid, dim3(256), 0,
                           ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
      else
        hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, false, 2, 5, 8>), grid, dim3(256), 0,
                           ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    } else {
      const dim3 gc(mb, (n + 255) / 256);
      const int* ord = nullptr;
      if (const spmm_status_t st = block_row_order(ctx, mb, gc.y, rowptr, &ord)) {
        timing_end(ctx, slot);
        return st;
      }
#ifdef SPMM_TUNING
      static const int env_tt = [] {
        const char* e = getenv("SPMM_CS16_TT");  // TUNING builds only
        return e ? atoi(e) : 0;
      }();
      const int ntt = env_tt && gc.y > 1 ? (int)gc.y : 0;
#else
      constexpr int ntt = 0;
#endif
      const dim3 gg = ntt ? dim3((unsigned)(8 * ((mb + 7) / 8) * ntt), 1) : gc;
#define CS16_LAUNCH(...)                                                                         \
  do {                                                                                           \
    if (crow)                                                                                    \
      hipLaunchKernelGGL((bsr16_f16_cs_kernel<true, 2, 4, 0, 48, __VA_ARGS__>), gg, dim3(64), 0, \
                         ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,   \
                         ord, masks, ntt);                                                       \
    else                                                                                         \
      hipLaunchKernelGGL((bsr16_f16_cs_kernel<false, 2, 4, 0, 48, __VA_ARGS__>), gg, dim3(64),   \
                         0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C,     \
                         ldc, ord, masks, ntt);                                                  \
  } while (0)
      if (msk) CS16_LAUNCH(true, true, 256, true);
      else if (lv == kBsr16F16Cs) CS16_LAUNCH(true, true);
      else CS16_LAUNCH(false, true);
#undef CS16_LAUNCH
    }
  } else if (bs == 16 && vec_ok) {
    const int waves = n <= 64 ? 1 : (n <= 128 ? 2 : 4);
    dim3 grid(mb, (n + 64 * waves - 1) / (64 * waves));
    SPMM_BSR_DISPATCH(bsr16_f16_mfma_kernel, SPMM_COMMA kBsr16F16Default, grid, dim3(64 * waves),
                      ctx->stream, rowd, brow, crow, mb, n, rowptr, colind, val, B, ldb, alpha,
                      beta, C, ldc);
  } else {
    dim3 grid(mb, (n + 63) / 64);
    hipLaunchKernelGGL(bsr_generic_kernel<_Float16>, grid, dim3(256), 0, ctx->stream, mb, n, bs,
                       rowd, rowptr, colind, val, B, ldb, brow, alpha, beta, C, ldc, crow);
  }
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsrmm_grouped_f32(spmm_context* ctx, int W, int mb, int n, int ngroups,
                                       const int* item_ptr, const int* rows,
                                       const unsigned* wmask, const float* afrag, const float* B,
                                       int ldb, float alpha, float beta, float* C, int ldc) {
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const int slot = timing_begin(ctx);
  const dim3 grid(ngroups, (n + 127) / 128);
  // stages and occupancy hint P * 10 + OCC (TUNING builds: SPMM_GRP32_VARIANT); chunks of
  // 32 block rows per XCD (SPMM_GRP_XM)
  int gv = 33, xm = 32 / W;
#ifdef SPMM_TUNING
  {
    static const int env = [] {
      const char* e = getenv("SPMM_GRP32_VARIANT");
      return e ? atoi(e) : 0;
    }();
    static const int env_xm = [] {
      const char* e = getenv("SPMM_GRP_XM");
      return e ? atoi(e) : -1;
    }();
    switch (env) {
      case 30: case 32: case 33: case 34: case 42: case 43: case 44: case 52: case 53: case 933:
        gv = env;
        break;
      default:
        break;
    }
    if (env_xm >= 0) xm = env_xm;
  }
#endif
#define GRP32_LAUNCH1(W_, P_, O_)                                                                \
  hipLaunchKernelGGL((bsr32_f32_grp_kernel<W_, P_, O_>), grid, dim3(64 * W_), 0, ctx->stream,    \
                     mb, n, item_ptr, rows, wmask, afrag, B, ldb, alpha, beta, C, ldc, xm)
#ifdef SPMM_TUNING
#define GRP32_LAUNCH(W_)                                                                         \
  do {                                                                                           \
    switch (gv) {                                                                                \
      case 30: GRP32_LAUNCH1(W_, 3, 0); break;                                                   \
      case 32: GRP32_LAUNCH1(W_, 3, 2); break;                                                   \
      case 34: GRP32_LAUNCH1(W_, 3, 4); break;                                                   \
      case 42: GRP32_LAUNCH1(W_, 4, 2); break;                                                   \
      case 43: GRP32_LAUNCH1(W_, 4, 3); break;                                                   \
      case 44: GRP32_LAUNCH1(W_, 4, 4); break;                                                   \
      case 52: GRP32_LAUNCH1(W_, 5, 2); break;                                                   \
      case 53: GRP32_LAUNCH1(W_, 5, 3); break;                                                   \
      case 933:  /* diagnostic: no MFMAs (wrong results) */                                    \
        hipLaunchKernelGGL((bsr32_f32_grp_kernel<W_, 3, 3, true>), grid, dim3(64 * W_), 0,       \
                           ctx->stream, mb, n, item_ptr, rows, wmask, afrag, B, ldb, alpha, beta, \
                           C, ldc, xm);                                                          \
        break;                                                                                   \
      default: GRP32_LAUNCH1(W_, 3, 3); break;                                                   \
    }                                                                                            \
  } while (0)
#else
#define GRP32_LAUNCH(W_) GRP32_LAUNCH1(W_, 3, 3)
#endif
  (void)gv;
  if (W == 4) GRP32_LAUNCH(4);
  else GRP32_LAUNCH(2);
#undef GRP32_LAUNCH
#undef GRP32_LAUNCH1
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_bsrmm_grouped_f16(spmm_context* ctx, int W, int mb, int n, int ngroups,
                                       const int* item_ptr, const int* rows,
                                       const unsigned* wmask, const unsigned* afrag,
                                       const uint16_t* B16, int ldb, float alpha, float beta,
                                       float* C, int ldc, bool crow) {
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const _Float16* B = reinterpret_cast<const _Float16*>(B16);
  const int slot = timing_begin(ctx);
  const int ntiles = (n + 255) / 256;
  // stages and occupancy hint: P * 10 + OCC, + 200 for two items per barrier (TUNING builds:
  // SPMM_GRP_VARIANT; SPMM_GRP_XM groups per XCD chunk)
  // chunks of 32 block rows per XCD, as the drop-in stream (xcd_block_row): neighbouring
  // groups share B rows in one L2 (W = 4: 3.10 -> 2.87 ms, profiles/r04e/grp_sweep.jsonl)
  // tiles together (ntt): a group's column tiles consecutive on one XCD, the later ones
  // reading the A fragments from L2: products stand-in 2.83 -> 2.62 ms, RCM 6.73 -> 6.38
  // (profiles/r04n/lines.jsonl)
  int gv = 33, xm = 32 / W, tt = 1;
#ifdef SPMM_TUNING
  {
    static const int env_tt = [] {
      const char* e = getenv("SPMM_GRP_TT");
      return e ? atoi(e) : -1;
    }();
    if (env_tt >= 0) tt = env_tt;
    static const int env = [] {
      const char* e = getenv("SPMM_GRP_VARIANT");
      return e ? atoi(e) : 0;
    }();
    static const int env_xm = [] {
      const char* e = getenv("SPMM_GRP_XM");
      return e ? atoi(e) : -1;
    }();
    // (4, 4) with two items per barrier is not offered: at W = 4 the allocator spills the A
    // fragments in flight (tools/isa_vmcnt.py --inflight). (3, 4) spilled with the vector row
    // loads (and faulted); with the scalar ones it audits clean
    // (every TUNING build is audited before it runs: tools/build_tuning.sh)
    switch (env) {
      case 30: case 33: case 32: case 42: case 43: case 52: case 53: case 23: case 24:
      case 243: case 262: case 263: case 1033: case 1043: case 34:
        gv = env;
        break;
      default:
        break;
    }
    if (env_xm >= 0) xm = env_xm;
  }
#endif
  const int ntt = tt && ntiles > 1 ? ntiles : 0;
  const dim3 grid = ntt ? dim3((unsigned)(8 * ((ngroups + 7) / 8) * ntt), 1)
                        : dim3((unsigned)ngroups, (unsigned)ntiles);
#define GRP_LAUNCH2(W_, P_, O_, IPB_, AL_)                                                       \
  do {                                                                                           \
    if (crow)                                                                                    \
      hipLaunchKernelGGL((bsr16_f16_grp_kernel<W_, P_, true, O_, IPB_, AL_>), grid,               \
                         dim3(64 * W_), 0, ctx->stream, mb, n, item_ptr, rows, wmask, afrag, B,   \
                         ldb, alpha, beta, C, ldc, xm, ngroups, ntt);                            \
    else                                                                                         \
      hipLaunchKernelGGL((bsr16_f16_grp_kernel<W_, P_, false, O_, IPB_, AL_>), grid,              \
                         dim3(64 * W_), 0, ctx->stream, mb, n, item_ptr, rows, wmask, afrag, B,   \
                         ldb, alpha, beta, C, ldc, xm, ngroups, ntt);                            \
  } while (0)
#define GRP_LAUNCH1(W_, P_, O_, IPB_) GRP_LAUNCH2(W_, P_, O_, IPB_, false)
#ifdef SPMM_TUNING
#define GRP_LAUNCH(W_)                                                                           \
  do {                                                                                           \
    switch (gv) {                                                                                \
      case 30: GRP_LAUNCH1(W_, 3, 0, 1); break;                                                  \
      case 32: GRP_LAUNCH1(W_, 3, 2, 1); break;                                                  \
      case 42: GRP_LAUNCH1(W_, 4, 2, 1); break;                                                  \
      case 43: GRP_LAUNCH1(W_, 4, 3, 1); break;                                                  \
      case 52: GRP_LAUNCH1(W_, 5, 2, 1); break;                                                  \
      case 53: GRP_LAUNCH1(W_, 5, 3, 1); break;                                                  \
      case 23: GRP_LAUNCH1(W_, 2, 3, 1); break;                                                  \
      case 24: GRP_LAUNCH1(W_, 2, 4, 1); break;                                                  \
      case 243: GRP_LAUNCH1(W_, 4, 3, 2); break;  /* two items per barrier */                    \
      case 262: GRP_LAUNCH1(W_, 6, 2, 2); break;                                                 \
      case 263: GRP_LAUNCH1(W_, 6, 3, 2); break;                                                 \
      case 34: GRP_LAUNCH1(W_, 3, 4, 1); break;  /* audited again after the scalar row loads */ \
      case 1033: GRP_LAUNCH2(W_, 3, 3, 1, true); break;  /* fragments through LDS */             \
      case 1043: GRP_LAUNCH2(W_, 4, 3, 1, true); break;                                          \
      default: GRP_LAUNCH1(W_, 3, 3, 1); break;                                                  \
    }                                                                                            \
  } while (0)
#else
#define GRP_LAUNCH(W_) GRP_LAUNCH1(W_, 3, 3, 1)
#endif
  (void)gv;
  if (W == 8) GRP_LAUNCH(8);
  else if (W == 4) GRP_LAUNCH(4);
  else GRP_LAUNCH(2);
#undef GRP_LAUNCH
#undef GRP_LAUNCH1
#undef GRP_LAUNCH2
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

}  // namespace spmm

extern "C" spmm_status_t spmm_bsr_small_path(spmm_handle_t handle, int* path) {
  if (!handle) return SPMM_STATUS_NOT_INITIALIZED;
  if (!path) return SPMM_STATUS_INVALID_VALUE;
  *path = handle->small_path;
  if (handle->small_path != 1) return SPMM_STATUS_SUCCESS;
  unsigned long long st[2] = {0, 0};
  hipError_t e = hipMemcpyAsync(st, handle->scratch, sizeof(st), hipMemcpyDeviceToHost,
                                handle->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(handle->stream);
  if (e != hipSuccess) return spmm::from_hip(e);
  if (SPMM_SGRP_PROBE && small_grp_gives_up(handle->small_path_bs, st[0], st[1])) *path = 2;
  return SPMM_STATUS_SUCCESS;
}
