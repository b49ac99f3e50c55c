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

// ---------------------------------------------------------------------------
// bs = 32 fp32, column-masked ("CM"): the LDS kernel above, but a B-panel row
// is fetched only when its column of the A block holds a nonzero, and an MFMA
// step runs only when one of its two k columns does. Blocks that csr2bsr cuts
// out of a sparse graph are mostly empty columns (19 % of panel rows used on
// the reddit stand-in, 23 % on products at bs = 32), and the full-panel
// kernel spends most of its HBM bytes and MFMA steps on them.
//
// The mask of a block needs its A values, so A runs ahead of B in its own
// ring (DA = D + 3 stages): at iteration k the waves
//   (a) OR the four per-wave partial masks of block k+D-1 (LDS, written at k-1),
//   (b) copy B(k+D-1): each lane of a masked-off row reads a 512-B zero row
//       instead (one L2-resident line set, same instruction count), so the
//       stage row holds exact zeros — an explicit zero of A then multiplies 0,
//       never stale data: explicit zeros inside a block act as structural
//       zeros (the CSR semantics of the same matrix; with finite B this is
//       the dense-block product exactly),
//   (c) compute this wave's partial mask of block k+D (8 rows: its own DMA
//       slot, one ds_read_b128, DPP OR inside 16-lane rows + 4 readlanes),
//   (d) copy A(k+DA-1),
//   (e) run block k's MFMAs, skipping quads / steps whose columns are empty.
// Copies per iteration: 4 (B) + 1 (A); B(k) and A(k+D) are both complete
// once at most 5 are outstanding, so one counted vmcnt(5) + lgkmcnt(0) and
// the raw barrier order everything, as in the kernel above.
// ---------------------------------------------------------------------------
// 1 KB of zeros: the source of masked-off B-panel rows (one 256-column fp32 row)
__device__ __attribute__((aligned(16))) float g_zero_row[256] = {0.f};

__device__ __forceinline__ int or_wave(int x) {
  // OR inside each 16-lane row (DPP row_ror 8 / 4 / 2 / 1), then across rows
  x |= __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
  x |= __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);
  x |= __builtin_amdgcn_update_dpp(0, x, 0x122, 0xF, 0xF, false);
  x |= __builtin_amdgcn_update_dpp(0, x, 0x121, 0xF, 0xF, false);
  return __builtin_amdgcn_readlane(x, 0) | __builtin_amdgcn_readlane(x, 16) |
         __builtin_amdgcn_readlane(x, 32) | __builtin_amdgcn_readlane(x, 48);
}

// DIAG (diagnostic builds only, wrong results): bit 0 no MFMA, bit 1 no B
// (every B row from the zero row), bit 2 every A copy from block k0.
template <bool CROW, int XM, int D = 3, int DA = D + 3, int DIAG = 0>
__global__ __launch_bounds__(256) void bsr32_f32_cm_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  static_assert(D >= 2 && D <= 4 && DA >= D + 2, "ring depths");
  // outstanding copies allowed at the top of iteration k with B(k) and A(k+D)
  // complete: 1 + 5(D-2) were issued after B(k), 5(DA-D-2) after A(k+D)
  constexpr int W = (1 + 5 * (D - 2)) < 5 * (DA - D - 2) ? 1 + 5 * (D - 2) : 5 * (DA - D - 2);
  constexpr int kA = 1024, kB = 32 * 128;  // floats per A block / B panel stage
  // one LDS array (A ring, B ring, partial masks [block & 3][wave])
  __shared__ __attribute__((aligned(16))) float smem[DA * kA + D * kB + 16];
  float* const sa = smem;
  float* const sb = smem + DA * kA;
  int* const part = reinterpret_cast<int*>(smem + DA * kA + D * kB);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = xcd_block_row(blockIdx.x, mb, XM);
  const int jt = blockIdx.y * 128;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  if (k0 >= k1) {
    const int j = jt + 32 * wv + (lane & 31);
    if (j < n)
      for (int e = 0; e < 16; ++e) {
        const size_t row = (size_t)br * 32 + 2 * e + (lane >> 5);
        float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
        *p = epi(0.f, alpha, beta, p);
      }
    return;
  }

  // A copy: lane l -> row 8w + l/8, LDS slot 4l holding logical chunk
  // (l%8) ^ swz(row) (same layout as bsr32_f32_lds_kernel).
  const int a_row = 8 * wv + (lane >> 3);
  const int a_chunk = (lane & 7) ^ ((a_row >> 1) & 7);
  const int a_src = a_row * 32 + 4 * a_chunk;
  const int b_col = min(jt + 4 * (lane & 31), n - 4);
  const int b_row = 8 * wv + (lane >> 5);
  const float* zsrc = g_zero_row + 4 * (lane & 31);
  auto wrapA = [](int s) { return s >= DA ? s - DA : s; };

  auto issue_a = [&](int k, int slot) {
    const int kk = (DIAG & 4) ? k0 : min(k, k1 - 1);
    __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)kk * 1024 + a_src),
                                     (lds_void_t)(sa + slot * kA + 256 * wv), 16, 0, 0);
  };
  auto issue_b = [&](int bc, unsigned mask, int slot) {
    const float* bsrc = B + ((size_t)bc * 32 + b_row) * ldb + b_col;
    float* dst = sb + slot * kB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool on = !(DIAG & 2) && ((mask >> (b_row + 2 * i)) & 1u);
      const float* src = on ? bsrc + (size_t)(2 * i) * ldb : zsrc;
      __builtin_amdgcn_global_load_lds((gbl_void_t)src,
                                       (lds_void_t)(dst + 128 * (8 * wv + 2 * i)), 16, 0, 0);
    }
  };
  // This wave's 8 rows of the A block in ring slot `slot` -> their column mask.
  auto partial = [&](int slot) -> int {
    const f32x4 x = *reinterpret_cast<const f32x4*>(sa + slot * kA + 256 * wv + 4 * lane);
    const int nib = (x[0] != 0.f) | ((x[1] != 0.f) << 1) | ((x[2] != 0.f) << 2) |
                    ((x[3] != 0.f) << 3);
    return or_wave(nib << (4 * a_chunk));
  };
  // Read through inline asm: the compiler's waitcnt pass would otherwise put
  // a vmcnt(0) on this LDS read (it cannot tell it from the DMA targets),
  // draining the copy pipeline every iteration. The partials it reads were
  // written with ds_write before the last barrier (lgkmcnt(0) there).
  const unsigned part_lds = (unsigned)reinterpret_cast<uintptr_t>(part);
  auto full = [&](int k) -> unsigned {
    int4 p;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(p) : "v"(part_lds + 16u * (unsigned)(k & 3)) : "memory");
    return (unsigned)__builtin_amdgcn_readfirstlane(p.x | p.y | p.z | p.w);
  };

  const int r = lane & 31, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  ColCursor cc(colind, k0, k1, lane);

  // Prologue: A(k0 .. k0+DA-2), masks of k0 .. k0+D-1, B(k0 .. k0+D-2).
#pragma unroll
  for (int d = 0; d < DA - 1; ++d) issue_a(k0 + d, d);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int d = 0; d < D; ++d) part[4 * ((k0 + d) & 3) + wv] = partial(d);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0));
  __builtin_amdgcn_s_barrier();
  unsigned mr[D - 1];  // masks of blocks k .. k+D-2
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    mr[d] = full(k0 + d);
    issue_b(cc.get(min(k0 + d, k1 - 1)), mr[d], d);
  }
  // B(k0) landed (4(D-2) copies follow it; the loop's W may exceed that)
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(W < 4 * (D - 2) ? W : 4 * (D - 2)));

  int sA = 0, sB = 0;  // ring slots of block k
  for (int k = k0; k < k1; ++k) {
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(W));
    __builtin_amdgcn_s_barrier();
    const unsigned mnew = full(k + D - 1);                                        // (a)
    issue_b(cc.get(min(k + D - 1, k1 - 1)), mnew, sB == 0 ? D - 1 : sB - 1);     // (b)
    part[4 * ((k + D) & 3) + wv] = partial(wrapA(sA + D));                       // (c)
    issue_a(k + DA - 1, sA == 0 ? DA - 1 : sA - 1);                              // (d)
    // (e) step s2 of half h uses column 16h + s2: pm bit s2 = either column set
    const unsigned pm = (DIAG & 1) ? 0u : (mr[0] | (mr[0] >> 16)) & 0xffffu;
    const float* stA = sa + sA * kA;
    const float* stB = sb + sB * kB + (16 * h) * 128 + 32 * wv + r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if ((pm >> (4 * q)) & 0xfu) {
        const int pc = (4 * h + q) ^ ((r >> 1) & 7);
        const f32x4 x = *reinterpret_cast<const f32x4*>(stA + r * 32 + 4 * pc);
        float fb[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) fb[s] = stB[(4 * q + s) * 128];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if ((pm >> (4 * q + s)) & 1u)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], fb[s], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int d = 0; d < D - 2; ++d) mr[d] = mr[d + 1];
    mr[D - 2] = mnew;
    sA = wrapA(sA + 1);
    sB = sB == D - 1 ? 0 : sB + 1;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // drain the clamped tail copies

  if constexpr (!CROW) {
    // Column-major C (cusparse layouts): the 32 x 128 tile goes through LDS so
    // each store instruction writes two whole 128-B column segments instead
    // of 64 scattered words.
    constexpr int kTs = 36;  // floats per tile column (32 rows, 16-B aligned)
    float* tile = smem;
    __syncthreads();  // every wave is past its last read of the rings
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(tile + (32 * wv + r) * kTs + 8 * g + 4 * h) =
          f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    __syncthreads();
    const size_t row = (size_t)br * 32 + r;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int jl = 2 * (4 * it + wv) + h;  // local column
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + r], alpha, beta, p);
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

// ---------------------------------------------------------------------------
// bs = 32 fp32, column-masked, four workgroups per CU ("CM4"): the CM kernel
// above in 40 960 B of LDS (2 A stages + 2 B stages), which is what a fourth
// workgroup per CU needs; the CM kernel's A ring (5 stages) and mask words
// hold it at three.
//  * A goes through VGPRs: each wave loads its own 8 rows of a block (one
//    dwordx4 per lane, the CM kernel's DMA layout) three blocks ahead and
//    writes them into the A stage one block before their MFMAs.
//  * No mask words: after a second barrier per block every wave reads the
//    whole next A block from LDS (4 x ds_read_b128 per lane) and reduces its
//    column mask itself.
// Per block k: barrier (B(k) landed, MFMA(k-1) done) -> write A(k+1) ->
// barrier -> mask(k+1) from LDS -> copy B(k+1) (zero row for empty columns)
// -> load A(k+4) -> MFMA(k) (steps of empty column pairs skipped). Numerics
// and semantics are the CM kernel's.
// ---------------------------------------------------------------------------
template <bool CROW, int XM>
__global__ __launch_bounds__(256) void bsr32_f32_cm4_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  constexpr int kA = 1024, kB = 32 * 128;  // floats per A / B stage
  __shared__ __attribute__((aligned(16))) float smem[2 * kA + 2 * kB];
  float* const sa = smem;
  float* const sb = smem + 2 * kA;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = xcd_block_row(blockIdx.x, mb, XM);
  const int jt = blockIdx.y * 128;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  if (k0 >= k1) {
    const int j = jt + 32 * wv + (lane & 31);
    if (j < n)
      for (int e = 0; e < 16; ++e) {
        const size_t row = (size_t)br * 32 + 2 * e + (lane >> 5);
        float* p = CROW ? C + row * ldc + j : C + (size_t)j * ldc + row;
        *p = epi(0.f, alpha, beta, p);
      }
    return;
  }

  // A: lane l holds row 8w + l/8, logical chunk (l%8) ^ swz(row), and writes it
  // to stage offset 256w + 4l (the CM kernel's swizzled layout).
  const int a_row = 8 * wv + (lane >> 3);
  const int a_src = a_row * 32 + 4 * ((lane & 7) ^ ((a_row >> 1) & 7));
  const int a_dst = 256 * wv + 4 * lane;
  const int b_col = min(jt + 4 * (lane & 31), n - 4);
  const int b_row = 8 * wv + (lane >> 5);
  const float* zsrc = g_zero_row + 4 * (lane & 31);
  f32x4 ra[3];  // A of blocks j = k + 1 .. k + 3 (register set (j - k0) % 3)
  // The A load must be the one vector-memory operation younger than the B
  // copies before it (the counted wait below keeps exactly one in flight).
  // The empty asm on its address is ordered after those copies (both have
  // side effects for the compiler), so the load cannot be hoisted above them;
  // the keep-alive after the loop stops hipcc from deleting the tail steps'
  // loads, whose values nothing reads (that deletion was the copy race, see
  // the wait in step()).
  typedef const __attribute__((address_space(1))) f32x4* gf32x4_ptr;  // a global load, not flat
  auto load_a = [&](int j) -> f32x4 {
    gf32x4_ptr p = (gf32x4_ptr)(val + (size_t)min(j, k1 - 1) * 1024 + a_src);
    asm volatile("" : "+v"(p));
    return *p;
  };
  auto put_a = [&](const f32x4& x, int slot) {
    *reinterpret_cast<f32x4*>(sa + slot * kA + a_dst) = x;
  };
  auto issue_b = [&](int bc, unsigned mask, int slot) {
    const float* bsrc = B + ((size_t)bc * 32 + b_row) * ldb + b_col;
    float* dst = sb + slot * kB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* src = ((mask >> (b_row + 2 * i)) & 1u) ? bsrc + (size_t)(2 * i) * ldb : zsrc;
      __builtin_amdgcn_global_load_lds((gbl_void_t)src,
                                       (lds_void_t)(dst + 128 * (8 * wv + 2 * i)), 16, 0, 0);
    }
  };
  // Column mask of the A block in `slot`, from the whole block: lane l reads
  // stage positions l + 64 i (row l/8 + 8 i, physical chunk l % 8). Through
  // inline asm: hipcc cannot tell the stage from the B copies' DMA targets
  // and would put a vmcnt(0) on these reads.
  const unsigned a_lds = (unsigned)reinterpret_cast<uintptr_t>(sa) + 16u * (unsigned)lane;
  auto mask_of = [&](int slot) -> unsigned {
    f32x4 x0, x1, x2, x3;
    const unsigned addr = a_lds + 4096u * (unsigned)slot;
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %4 offset:1024\n\t"
        "ds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)  // early clobber: the address
        : "v"(addr)                                    // must outlive the first read
        : "memory");
    const f32x4 xs[4] = {x0, x1, x2, x3};
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lc = (lane & 7) ^ (((lane >> 4) + 4 * i) & 7);
      const int nib = (xs[i][0] != 0.f) | ((xs[i][1] != 0.f) << 1) | ((xs[i][2] != 0.f) << 2) |
                      ((xs[i][3] != 0.f) << 3);
      m |= nib << (4 * lc);
    }
    return (unsigned)or_wave(m);
  };

  const int r = lane & 31, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  ColCursor cc(colind, k0, k1, lane);

  // Prologue: A(k0 .. k0+2) into registers, A(k0) into stage 0, its mask,
  // B(k0), then A(k0+3) into the registers A(k0) left.
  ra[0] = load_a(k0);
  ra[1] = load_a(k0 + 1);
  ra[2] = load_a(k0 + 2);
  put_a(ra[0], 0);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(63));
  __builtin_amdgcn_s_barrier();
  unsigned mk = mask_of(0);
  issue_b(cc.get(k0), mk, 0);
  ra[0] = load_a(k0 + 3);

  // Block k uses A / B stage (k - k0) & 1; its A came from register set
  // (k - k0) % 3. The loop runs in rounds of 3 blocks with no exit inside
  // (an exit merging back into the loop head makes hipcc drain the register
  // ring there); the remainder runs after it.
  auto step = [&](auto U, int k) {
    constexpr int u = decltype(U)::value;  // (k - k0) % 3
    const int sl = (k - k0) & 1;
    // B(k) landed, MFMA(k-1) retired: every operation but the youngest, the
    // A(k+3) load issued right after the B(k) copies, is complete.
    // History: this wait was vmcnt(1) from the start, but
    // hipcc deleted the A loads of the two tail steps (their values are
    // never read), so in the second tail step the one operation the wait left
    // in flight was the last B copy of the row's last block, and the waves
    // reading it early lost one term a_rc * B[c] (block rows with
    // (k1 - k0) % 3 == 2). load_a pins the load in place and the keep-alive
    // after the loop keeps it; tests/test_isa_waits.py checks the emitted
    // window of every such wait.
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(1));
    __builtin_amdgcn_s_barrier();
    put_a(ra[(u + 1) % 3], sl ^ 1);                       // A(k+1)
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(63));
    __builtin_amdgcn_s_barrier();
    const unsigned m1 = mask_of(sl ^ 1);
    issue_b(cc.get(min(k + 1, k1 - 1)), m1, sl ^ 1);      // B(k+1)
    ra[(u + 1) % 3] = load_a(k + 4);                      // A(k+4)
    const unsigned pm = (mk | (mk >> 16)) & 0xffffu;
    const float* stA = sa + sl * kA;
    const float* stB = sb + sl * kB + (16 * h) * 128 + 32 * wv + r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if ((pm >> (4 * q)) & 0xfu) {
        const int pc = (4 * h + q) ^ ((r >> 1) & 7);
        const f32x4 x = *reinterpret_cast<const f32x4*>(stA + r * 32 + 4 * pc);
        float fb[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) fb[s] = stB[(4 * q + s) * 128];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if ((pm >> (4 * q + s)) & 1u)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], fb[s], acc, 0, 0, 0);
      }
    }
    mk = m1;
  };
  const int kfull = k0 + (k1 - k0) / 3 * 3;
  for (int kb = k0; kb < kfull; kb += 3) {
    step(std::integral_constant<int, 0>{}, kb);
    step(std::integral_constant<int, 1>{}, kb + 1);
    step(std::integral_constant<int, 2>{}, kb + 2);
  }
  if (kfull < k1) step(std::integral_constant<int, 0>{}, kfull);
  if (kfull + 1 < k1) step(std::integral_constant<int, 1>{}, kfull + 1);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // drain the clamped tail copies
  asm volatile("" ::"v"(ra[0]), "v"(ra[1]), "v"(ra[2]));  // keep every A load

  if constexpr (!CROW) {
    constexpr int kTs = 36;  // floats per tile column (32 rows, 16-B aligned)
    float* tile = smem;
    __syncthreads();  // every wave is past its last read of the stages
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(tile + (32 * wv + r) * kTs + 8 * g + 4 * h) =
          f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    __syncthreads();
    const size_t row = (size_t)br * 32 + r;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int jl = 2 * (4 * it + wv) + h;  // local column
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + r], alpha, beta, p);
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
      float* p = C + row * ldc + jcol;
      *p = epi(acc[4 * g + e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 32, column stream (CS; ROW blocks, row-major B): one wave per (block
// row, 128 output columns), no barriers. The block-level kernels above keep
// four waves in step on one block at a time, so every block costs a barrier
// chain and a B stage sized for 32 rows although 73-82 % of the blocks on
// the stand-ins hold one nonzero column. Here a wave streams the block row as
// a sequence of ITEMS, one per pair of nonzero columns (c0, c1) of a block
// (a single column when the count is odd):
//  * A ring (NA slots x 4 KB of LDS): block k + DA is copied by LDS-DMA (4 x
//    global_load_lds_dwordx4, the XOR-swizzled layout of the kernels above)
//    when the producer reaches block k. Its column mask comes from 8
//    ds_read2st64_b32 (lane l reads column l % 32 of 16 rows, rows r and
//    r + 16 share a swizzle), a masked OR of the 16 values and one ballot:
//    no cross-lane reduction.
//  * Item ring (P slots x 1 KB of LDS): an item's two B rows (512 B each,
//    lanes 0-31 row c0, lanes 32-63 row c1) are one global_load_lds_dwordx4;
//    its two A columns are read from the A slot into registers at issue time
//    (a static ring of 2P VGPRs: the loop is unrolled P times), so the A slot
//    is free as soon as the block's last item is issued.
//  * The item issued P steps earlier is consumed: two ds_read_b64 and
//    v_mfma_f32_32x32x1_2b_f32 per column and 64-column half. The 2-block
//    form takes one k per MFMA, so a single column costs 2 MFMAs (128 cycles)
//    and a pair 4 — the 32x32x2 step of a lone column is half zeros.
// Waits: every vector-memory operation of the loop is an LDS-DMA copy (B rows,
// A blocks) and they retire in issue order (MI355X_MICROARCH.md §vmcnt), so
// the wave keeps a count of copies issued; each slot records the count at
// its copy and the wait for it is vmcnt(q), q the largest ladder value not
// above the number of younger copies (wait_vm_older). All LDS reads are inline
// asm that end in lgkmcnt(0): their results exist when the compiler sees
// them, and hipcc puts no conservative vmcnt(0) before them.
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
__device__ __forceinline__ int block_row_key(int i, const int* __restrict__ rowptr,
                                             const int* __restrict__ crp, int m) {
  const int nb = rowptr[i + 1] - rowptr[i];
  if (!crp) return min(nb, 1023);
  const int rem = crp[min(32 * i + 32, m)] - crp[32 * i];
  return min((32 * nb + rem) >> 3, 1023);
}
__global__ __launch_bounds__(1024) void block_row_order_kernel(int mb, const int* __restrict__ rowptr,
                                                               const int* __restrict__ crp, int m,
                                                               int* __restrict__ order) {
  __shared__ int cnt[1024];
  const int t = threadIdx.x;
  cnt[t] = 0;
  __syncthreads();
  for (int i = t; i < mb; i += 1024) atomicAdd(&cnt[1023 - block_row_key(i, rowptr, crp, m)], 1);
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
    order[atomicAdd(&cnt[1023 - block_row_key(i, rowptr, crp, m)], 1)] = i;
}

template <bool CROW, int XM, int P, int NA>
__global__ __launch_bounds__(64) void bsr32_f32_cs_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  static_assert(NA >= 2 && NA <= 4 && P >= 2 && P <= 16, "ring depths");
  constexpr int DA = NA - 1;  // A blocks in flight ahead of the producer's block
  constexpr int kRings = NA * 1024 + P * 256;  // floats
  // (column-major C reuses the LDS for a 128 x 36-float tile)
  __shared__ __attribute__((aligned(16))) float smem[CROW || kRings >= 128 * 36 ? kRings : 128 * 36];
  const int lane = threadIdx.x;
  const int j = lane & 31, h = lane >> 5;
  const int br = xcd_block_row(blockIdx.x, mb, XM);
  const int jt = blockIdx.y * 128;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const unsigned lds_a = (unsigned)reinterpret_cast<uintptr_t>(smem);
  const unsigned lds_b = lds_a + NA * 4096u;

  // A copy q (0..3) of a block: lane l -> row 8q + l/8, logical chunk
  // (l % 8) ^ ((row / 2) % 8); rows of copies q and q + 2 share the swizzle.
  int a_src[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * q + (lane >> 3);
    a_src[q] = r * 32 + 4 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  auto issue_a = [&](int kk, int slot) {
    const float* src = val + (size_t)kk * 1024;
    float* dst = smem + slot * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(src + a_src[q & 1] + 512 * (q >> 1)),
                                       (lds_void_t)(dst + 256 * q), 16, 0, 0);
  };
  // Mask reads: rows 2i + h and 2i + h + 16 (i = 0..7), column j; row r holds
  // column c at byte r*128 + 16*((c/4) ^ ((r/2) % 8)) + 4*(c % 4).
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
  // A column c of the block in `slot`, lane (j, h): A[j][c]
  const unsigned a_row = (unsigned)(j * 128);
  const int a_sw = (j >> 1) & 7;
  auto a_cols = [&](int slot, int c0, int c1, float& x0, float& x1) {
    const unsigned base = lds_a + 4096u * (unsigned)slot + a_row;
    const unsigned p0 = base + 16u * (unsigned)((c0 >> 2) ^ a_sw) + 4u * (unsigned)(c0 & 3);
    const unsigned p1 = base + 16u * (unsigned)((c1 >> 2) ^ a_sw) + 4u * (unsigned)(c1 & 3);
    asm volatile(
        "ds_read_b32 %0, %2\n\t"
        "ds_read_b32 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1)
        : "v"(p0), "v"(p1)
        : "memory");
  };
  const int bcol = min(jt + 4 * j, n - 4);
  const unsigned b_rd = lds_b + 16u * (unsigned)j + 8u * (unsigned)h;

  f32x32 u0, u1;  // MFMA halves u = 0, 1 (output columns 4j + 2b + u)
#pragma unroll
  for (int e = 0; e < 32; ++e) u0[e] = u1[e] = 0.f;

  int nis = 0;  // copies issued by this wave
  int ast[DA];  // copy count at each A block in flight (k+1 .. k+DA)
  int aslot = NA - 1;
  int k = k0 - 1;
  unsigned m = 0;
  bool more = true;
  int bc = 0, bcn = k0 < k1 ? colind[k0] : 0;
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
  int kind[P], stamp[P];
  float ra0[P], ra1[P];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    kind[s] = 0;
    stamp[s] = 0;
    ra0[s] = ra1[s] = 0.f;
  }

  for (;;) {
    const bool fin = !more;
#pragma unroll
    for (int s = 0; s < P; ++s) {
      // consume the item issued P steps ago
      if (kind[s]) {
        wait_vm_older(nis - stamp[s]);
        f32x2 b0, b1;
        asm volatile(
            "ds_read_b64 %0, %2 offset:%3\n\t"
            "ds_read_b64 %1, %2 offset:%4\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(b0), "=&v"(b1)
            : "v"(b_rd), "n"(s * 1024), "n"(s * 1024 + 512)
            : "memory");
        u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(ra0[s], b0[0], u0, 0, 0, 0);
        u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(ra0[s], b0[1], u1, 0, 0, 0);
        if (kind[s] == 2) {
          u0 = __builtin_amdgcn_mfma_f32_32x32x1f32(ra1[s], b1[0], u0, 0, 0, 0);
          u1 = __builtin_amdgcn_mfma_f32_32x32x1f32(ra1[s], b1[1], u1, 0, 0, 0);
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
          ++k;
          aslot = aslot + 1 == NA ? 0 : aslot + 1;
          wait_vm_older(nis - ast[0]);  // A(k) landed
#pragma unroll
          for (int d = 0; d + 1 < DA; ++d) ast[d] = ast[d + 1];
          bc = bcn;
          bcn = colind[min(k + 1, k1 - 1)];
          m = mask_of(aslot);
          if (k + DA < k1) {
            issue_a(k + DA, aslot + DA >= NA ? aslot + DA - NA : aslot + DA);
            nis += 4;
            ast[DA - 1] = nis;
          } else {
            ast[DA - 1] = -64;
          }
        }
        if (m != 0u) {
          const int c0 = __builtin_ctz(m);
          m &= m - 1u;
          int c1 = c0;
          kind[s] = 1;
          if (m != 0u) {
            c1 = __builtin_ctz(m);
            m &= m - 1u;
            kind[s] = 2;
          }
          a_cols(aslot, c0, c1, ra0[s], ra1[s]);
          const float* src = B + (size_t)(bc * 32 + (h ? c1 : c0)) * ldb + bcol;
          __builtin_amdgcn_global_load_lds((gbl_void_t)src, (lds_void_t)(smem + NA * 1024 + s * 256),
                                           16, 0, 0);
          stamp[s] = ++nis;
        }
      }
    }
    // keeps the accumulators in AGPRs across the loop (else hipcc parks one
    // in VGPRs at the loop head and copies it back before the first MFMA)
    asm volatile("" : "+a"(u0), "+a"(u1));
    if (fin) break;
  }

  // Epilogue. Lane (j, h), accumulator element e: row (e % 4) + 8 (e / 4) + 4h
  // of the block row; u0 / u1 block 0 -> columns 4j, 4j + 1, block 1 ->
  // 4j + 2, 4j + 3.
  if constexpr (CROW) {
    const int col = jt + 4 * j;
    if (col >= n) return;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      f32x4* p = reinterpret_cast<f32x4*>(C + row * ldc + col);
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
    // column-major C: the tile goes through LDS as [column][row] (36-float
    // columns), then each store writes two 128-B column segments
    constexpr int kTs = 36;
    float* tile = smem;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      tile[(4 * j) * kTs + row] = u0[e];
      tile[(4 * j + 1) * kTs + row] = u1[e];
      tile[(4 * j + 2) * kTs + row] = u0[16 + e];
      tile[(4 * j + 3) * kTs + row] = u1[16 + e];
    }
    __builtin_amdgcn_s_waitcnt(0);
    const size_t row = (size_t)br * 32 + j;
    for (int it = 0; it < 64; ++it) {
      const int jl = 2 * it + h;
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + j], alpha, beta, p);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 32, column stream with register items (CS2). The CS kernel above
// stages an item's two B rows in an LDS ring (8 KB of its 20 KB), which holds
// it to eight waves per CU, and reads them back with one more LDS round trip
// per item. Here the rows go straight into registers: per item one or two
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
// DIAG (diagnostic builds, wrong results, timing only): bit 0 no MFMA, bit 1
// every B row from the L2-resident zero row, bit 2 every A copy from block k0.
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
template <bool CROW, int XM, int P, int NA, int DIAG = 0, bool O32 = false, bool PK = false,
          bool ANT = false>
__global__ __launch_bounds__(64) void bsr32_f32_cs2_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, const float* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc, const int* __restrict__ order,
    const int4* __restrict__ segs = nullptr, float* __restrict__ part = nullptr) {
  static_assert(NA >= 2 && NA <= 4 && P >= 2 && P <= 16, "ring depths");
  constexpr int DA = NA - 1;  // A blocks in flight ahead of the producer's block
  // (column-major C reuses the LDS for a 128 x 36-float tile)
  __shared__ __attribute__((aligned(16)))
  float smem[CROW || NA * 1024 >= 128 * 36 ? NA * 1024 : 128 * 36];
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
    k0 = rowptr[br];
    k1 = rowptr[br + 1];
  }
  const int jt = blockIdx.y * 128;
  const unsigned lds_a = (unsigned)reinterpret_cast<uintptr_t>(smem);

  int a_src[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * q + (lane >> 3);
    a_src[q] = r * 32 + 4 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  auto issue_a = [&](int kk, int slot) {
    const float* src = val + (size_t)((DIAG & 4) ? k0 : kk) * 1024;
    float* dst = smem + slot * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(src + a_src[q & 1] + 512 * (q >> 1)),
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
  const unsigned boff = 4u * (unsigned)min(jt + 4 * j + 2 * h, n - 2);  // byte offset in a row
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
  auto load_cols = [&](int kstart) {
    const unsigned off = 4u * (unsigned)min(kstart + lane, k1 - 1);
    asm volatile("global_load_dword %0, %1, %2" : "=&v"(cnext) : "v"(off), "s"(colind) : "memory");
    cstamp = ++nis;
  };
  if (k0 < k1) load_cols(k0);
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
  int kind[P], stamp[P];
  float ra0[P], ra1[P];  // in flight: asm-only registers
  f32x2 rb0[P], rb1[P];  // in flight: asm-only registers
#pragma unroll
  for (int s = 0; s < P; ++s) {
    kind[s] = 0;
    stamp[s] = -64;
    ra0[s] = ra1[s] = 0.f;
    rb0[s] = rb1[s] = f32x2{0.f, 0.f};
  }

  // next block: its column chunk, A landed, its mask, the copy of block k + DA
  auto advance = [&]() {
    ++k;
    aslot = aslot + 1 == NA ? 0 : aslot + 1;
    const int kr = k - k0;
    if ((kr & 63) == 0) {  // next block-column chunk
      asm volatile(SPMM_VM_LADDER("%1") "v_mov_b32 %0, %2"
                   : "=&v"(ccur)
                   : "s"(nis - cstamp), "v"(cnext)
                   : "scc", "memory");
      if (k + 64 < k1) load_cols(k + 64);
    }
    const int bc = __builtin_amdgcn_readlane(ccur, kr & 63);
    bblk = (DIAG & 2) ? reinterpret_cast<const char*>(g_zero_row)
                      : reinterpret_cast<const char*>(B) + (size_t)bc * 32 * ldb4;
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
  // LDS address of this lane's A value of column c of the current block
  auto acol = [&](int c) -> unsigned {
    return lds_a + 4096u * (unsigned)aslot + a_row + 16u * (unsigned)((c >> 2) ^ a_sw) +
           4u * (unsigned)(c & 3);
  };
  // B row c of the current block's panel into r (in flight: asm-only register)
  auto load_row = [&](f32x2& r, int c) {
    if constexpr (O32)
      asm volatile("global_load_dwordx2 %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff + (unsigned)c * ldb4u), "s"(bblk)
                   : "memory");
    else
      asm volatile("global_load_dwordx2 %0, %1, %2"
                   : "=&v"(r)
                   : "v"(boff), "s"(bblk + ((DIAG & 2) ? 0 : (size_t)c * ldb4))
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
      {
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
        if (!(DIAG & 1) && kind[s]) {
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
            asm volatile("ds_read_b32 %0, %1" : "=&v"(ra0[s]) : "v"(acol(c0)) : "memory");
            load_row(rb0[s], c0);
            kind[s] = 1;
            while (m == 0u && k + 1 < k1) advance();  // pair with the next block's first column
            if (m != 0u) {
              const int c1 = __builtin_ctz(m);
              m &= m - 1u;
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
            asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3"
                         : "=&v"(ra0[s]), "=&v"(ra1[s])
                         : "v"(acol(c0)), "v"(acol(c1))
                         : "memory");
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
    asm volatile("" : "+a"(u0), "+a"(u1));
    if (fin) break;
  }
  // nothing is in flight after the last round; the full wait makes that
  // visible to the register check (tests/test_isa_waits.py)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+a"(u0), "+a"(u1) : : "memory");

  if constexpr (CROW) {
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
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const size_t row = (size_t)br * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      f32x4* p = reinterpret_cast<f32x4*>(C + row * ldc + col);
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
    float* tile = smem;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
      tile[(4 * j) * kTs + row] = u0[e];
      tile[(4 * j + 1) * kTs + row] = u1[e];
      tile[(4 * j + 2) * kTs + row] = u0[16 + e];
      tile[(4 * j + 3) * kTs + row] = u1[16 + e];
    }
    __builtin_amdgcn_s_waitcnt(0);
    const size_t row = (size_t)br * 32 + j;
    for (int it = 0; it < 64; ++it) {
      const int jl = 2 * it + h;
      if (jt + jl < n) {
        float* p = C + (size_t)(jt + jl) * ldc + row;
        *p = epi(tile[jl * kTs + j], alpha, beta, p);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16, LDS-staged (ROW blocks, row-major B), fp32 or fp16 A/B: the shipped
// bs = 16 kernels where the layout allows it. Same scheme as the bs = 32
// one: a workgroup (4 waves, 256 output columns, 64 per wave) copies each
// block's A (16 x 16) and B panel (16 rows x 256 columns) into LDS with
// global_load_lds_dwordx4, D - 1 blocks ahead, one raw barrier per block.
//  * fp32: v_mfma_f32_16x16x4_f32 with k = 4g + s (lane group g = lane/16), so
//    a lane's A fragment is one ds_read_b128; B by ds_read_b32.
//  * fp16: v_mfma_f32_16x16x16_f16 (one block per instruction); the B
//    fragment (4 consecutive k of one column) comes from the row-major panel
//    through ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group,
//    delivered column-wise) — the fragment-shaped 2-byte global loads of the
//    kernel below are gone.
// B panel rows are 16-byte-chunk XOR-swizzled (source side and read side) so
// the reads are bank-conflict-free.
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
// One ds_read_b64 and its wait, for an LDS read hipcc would otherwise fence
// with vmcnt(0) (same reason as above).
__device__ __forceinline__ f16x4 ds_read_f16x4(unsigned a) {
  f16x4 r;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
  return r;
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)reinterpret_cast<uintptr_t>(p);
}

template <typename T>
__device__ __forceinline__ int bsr16_swz(int row) {
  return sizeof(T) == 2 ? 2 * (row & 7) : 4 * ((row >> 2) & 1);
}

template <typename T, bool CROW, int D, bool XCD = false>
__global__ __launch_bounds__(256) void bsr16_lds_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const T* __restrict__ val, const T* __restrict__ B, int ldb, float alpha, float beta,
    float* __restrict__ C, int ldc) {
  constexpr int kEpc = 16 / sizeof(T);             // elements per 16-B chunk
  constexpr int kA = 256 * sizeof(T);              // A block bytes
  constexpr int kRowB = 256 * sizeof(T);           // B panel row bytes (256 columns)
  constexpr int kStage = kA + 16 * kRowB;          // bytes per stage
  constexpr int kRpi = 1024 / kRowB;               // B rows per copy instruction (1 or 2)
  constexpr int kCpr = kRowB / 16;                 // chunks per B row (64 or 32)
  __shared__ __attribute__((aligned(16))) char smem[D * kStage];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int br = xcd_block_row(blockIdx.x, mb, XCD ? 1 : 0);  // XCD-contiguous option
  const int jt = blockIdx.y * 256;
  const int g = lane >> 4, c16 = lane & 15;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  if (k0 >= k1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = jt + 64 * wv + 16 * t + c16;
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

  // Copy sources of this wave: A rows 4w .. 4w+3 (lanes 0 .. kA/64 - 1, 16 B
  // each, contiguous in the block) and B panel rows 4w .. 4w+3.
  const bool a_lane = lane < kA / 64;
  const int a_src = (4 * wv) * 16 + lane * kEpc;
  int b_src[4 / kRpi];
#pragma unroll
  for (int i = 0; i < 4 / kRpi; ++i) {
    const int row = 4 * wv + i * kRpi + lane / kCpr;
    const int c = (lane % kCpr) ^ bsr16_swz<T>(row);
    b_src[i] = row * ldb + min(jt + c * kEpc, n - kEpc);
  }
  auto issue = [&](int k, int bc, int st) {
    const int kk = min(k, k1 - 1);
    char* stage = smem + st * kStage;
    if (a_lane)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)kk * 256 + a_src),
                                       (lds_void_t)(stage + wv * (kA / 4)), 16, 0, 0);
    const T* bp = B + (size_t)bc * 16 * ldb;
#pragma unroll
    for (int i = 0; i < 4 / kRpi; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_t)(bp + b_src[i]),
                                       (lds_void_t)(stage + kA + (4 * wv + i * kRpi) * kRowB),
                                       16, 0, 0);
  };
  constexpr int kIssued = 1 + 4 / kRpi;  // copy instructions per wave and block

  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  ColCursor cc(colind, k0, k1, lane);
#pragma unroll
  for (int d = 0; d < D - 1; ++d) issue(k0 + d, cc.get(min(k0 + d, k1 - 1)), d);

  int st = 0;
  for (int k = k0; k < k1; ++k) {
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(kIssued * (D - 2)));
    __builtin_amdgcn_s_barrier();
    issue(k + D - 1, cc.get(min(k + D - 1, k1 - 1)), st == 0 ? D - 1 : st - 1);
    const char* stage = smem + st * kStage;
    const char* bpan = stage + kA;
    if constexpr (sizeof(T) == 2) {
      // A: row c16, k = 4g .. 4g+3. B: group g reads rows 4g .. 4g+3 transposed.
      const f16x4 fa = *reinterpret_cast<const f16x4*>(stage + c16 * 32 + 8 * g);
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int row = 4 * g + q;
      unsigned ad[4];
      f16x4 fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = 64 * wv + 16 * t + 4 * p;
        ad[t] = lds_addr(bpan + row * kRowB + (((col >> 3) ^ bsr16_swz<T>(row)) << 4) + (col & 7) * 2);
      }
      ds_read_tr16_n(fb, ad);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa, fb[t], acc[t], 0, 0, 0);
    } else {
      // A: row c16, k = 4g + s (s = 0..3) -> one 16-B read.
      const f32x4 fa = *reinterpret_cast<const f32x4*>(stage + c16 * 64 + 16 * g);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int row = 4 * g + s2;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int col = 64 * wv + 16 * t + c16;
          const int off = row * kRowB + (((col >> 2) ^ bsr16_swz<T>(row)) << 4) + (col & 3) * 4;
          const float fb = *reinterpret_cast<const float*>(bpan + off);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s2], fb, acc[t], 0, 0, 0);
        }
      }
    }
    st = st == D - 1 ? 0 : st + 1;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));

#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int j = jt + 64 * wv + 16 * t + c16;
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
// bs = 16, column-masked: the bs = 32 CM scheme on bsr16_lds_kernel's layout
// (4 waves, 256 output columns, A block row-major in LDS, B panel rows
// 16-B-chunk swizzled). Only B rows of nonzero A columns are fetched (41 % on
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
  auto full = [&](int k) -> unsigned {  // inline asm: see bsr32_f32_cm_kernel
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
//    copy (the run-time vmcnt ladder of bsr32_f32_cs_kernel: every
//    vector-memory operation of the loop is counted), 16 ds_read_b64_tr_b16
//    under one lgkmcnt wait, 16 MFMAs into 16 accumulator tiles.
// ---------------------------------------------------------------------------
// DIAG (diagnostic builds, wrong results, timing only): bit 0 no MFMA, bit 1 every B row
// from the L2-resident zero row, bit 2 every A copy from the row's first block, bit 3 no
// item copies at all (the stage is read stale).
constexpr int kIsRec = 576;  // item record: 16 B-row indices + the 16 x 16 fp16 A fragment
// BUILD (the item-stream builder, bsr16_f16_is_kernel's first launch): the same walk over
// the block row, once for all columns; each emitted item is stored as a 576-B record
// (kIsRec) instead of being copied and multiplied, and nitems[br] gets the item count.
// FLC (full-line copies): the item's B rows are copied one 256-B half row per LDS-DMA
// (global_load_lds_dword, 32 per item) into rows of 528 B, so every copy reads two whole
// 128-B lines (the 16-B form reads 16 half lines per copy, the other halves one copy
// later) and the transposed reads (16 rows at a 528-B pitch) stay conflict-free.
template <bool CROW, int P, int NA, int DA, int COLS = 256, int CAP = 64, int DIAG = 0,
          bool BUILD = false, bool FLC = false, bool FLR = false, bool TT = false>
__global__ __launch_bounds__(64) void bsr16_f16_cs_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const _Float16* __restrict__ val, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, const int* __restrict__ order,
    char* __restrict__ items, int* __restrict__ nitems) {
  // the pair copied at block kr (blocks kr + DA + 2, + 3) overwrites blocks
  // kr + DA + 2 - NA, + 3 - NA, which must be read already (< kr)
  static_assert((NA & (NA - 1)) == 0 && DA % 2 == 0 && NA >= DA + 4 && P >= 2 && P <= 6,
                "ring depths");
  static_assert(COLS == 128 || COLS == 256, "column tile");
  // pending-list capacity: 64 entries, or 48 (a smaller A-fragment buffer: 8 waves per CU
  // with NA = 4); a pair of blocks adds at most 32 to at most 15 pending
  static_assert(CAP == 64 || CAP == 48, "pending capacity");
  constexpr int kT = COLS / 16;           // 16-column MFMA tiles per wave
  constexpr int kCopies = COLS / 32;      // copies per item (16 rows x 4 chunks each)
  static_assert(!FLC || COLS == 256, "full-line copies: 256 columns");
  static_assert(!FLR || (COLS == 256 && !FLC), "two-row copies: 256 columns");
  constexpr int kRowP = 528;              // FLC row pitch
  constexpr int kStage = FLC ? 16 * kRowP : 16 * COLS * 2;  // one item: 16 B rows x COLS fp16
  // A-fragment buffer row: CAP entries + a dummy entry (index CAP) + pad; 136 / 104 B rows put
  // the four row groups' writes in different banks
  constexpr int kAbRow = CAP == 64 ? 136 : 104;
  constexpr int kAbuf = NA * 512;   // offset of the A-fragment buffer
  constexpr int kStg = kAbuf + 16 * kAbRow;  // offset of the item stages
  constexpr int kLds = BUILD ? kStg : kStg + P * kStage;
  static_assert(BUILD || kLds >= COLS * 16 * 4, "column-major C tile fits");
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int lane = threadIdx.x;
  const int g = lane >> 4, r16 = lane & 15, h = lane >> 5;
  // TT: the column tiles of one block row are neighbouring waves of one XCD
  // (a one-dimensional grid of mb x tiles waves, tiles fastest inside each
  // XCD chunk), so the second tile's A blocks and block columns come from the
  // XCD's L2 while the first tile's wave is still streaming them.
  int br, tile;
  if constexpr (TT) {
    const int nt = (n + COLS - 1) / COLS;
    if (order) {
      br = order[blockIdx.x / nt];
      tile = blockIdx.x % nt;
    } else {
      const int w = xcd_block_row(blockIdx.x, mb * nt, 32 * nt);
      br = w / nt;
      tile = w % nt;
    }
  } else {
    br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, 32);
    tile = blockIdx.y;
  }
  int nit = 0;  // BUILD: items stored
  const int jt = tile * COLS;
  const int k0 = rowptr[br], k1 = rowptr[br + 1];
  const unsigned lds0 = lds_addr(smem);
  const unsigned abuf = lds0 + kAbuf;

  // copy j: lane L loads chunk 4j + L / 16 of its row (columns jt + 8 (4j + L / 16) ..)
  unsigned boff[kCopies];
#pragma unroll
  for (int j = 0; j < kCopies; ++j) boff[j] = 2u * (unsigned)min(jt + 8 * (4 * j + g), n - 8);
  const size_t ldb2 = (size_t)ldb * 2;
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 2 * (size_t)jt;
  // transposed B reads: lane (g, q = (lane >> 2) & 3, p = lane & 3) reads row 4g + q,
  // columns 16t + 4p .. + 3: chunk 2t + p / 2 at byte 8 (p & 1); t by immediate offset
  const unsigned tro =
      FLC ? lds0 + kStg + (unsigned)kRowP * (4 * g + ((lane >> 2) & 3)) + 8u * (lane & 3)
          : lds0 + kStg + 256u * ((lane & 3) >> 1) + 16u * (4 * g + ((lane >> 2) & 3)) +
                8u * (lane & 1);
  // FLR: copy j brings item rows 2j (lanes 0-31) and 2j + 1 (lanes 32-63) whole, so each copy
  // reads 8 whole 128-B lines; lane k of row R loads chunk (k - R) & 31, which puts chunk c of
  // row R at 16-B slot (c + R) & 31 of its 512-B stage row: the 16 rows of one chunk sit in 16
  // different bank slots, and the transposed reads take one address per t (tra).
  unsigned boffr[8], tra[16];
  if constexpr (FLR) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      boffr[j] = 2u * (unsigned)min(jt + 8 * (((lane & 31) - 2 * j - (lane >> 5)) & 31), n - 8);
    const int R = 4 * g + ((lane >> 2) & 3);
#pragma unroll
    for (int t = 0; t < 16; ++t)
      tra[t] = lds0 + kStg + 512u * R + 16u * ((2 * t + ((lane & 3) >> 1) + R) & 31) + 8u * (lane & 1);
  }
  // FLC: 4 B (2 columns) per lane and copy, the row's two halves
  const unsigned boffl = 2u * (unsigned)min(jt + 2 * lane, n - 2);
  const unsigned boffh = 2u * (unsigned)min(jt + 128 + 2 * lane, n - 2);

  int nis = 0;  // vector-memory operations issued by this wave
  // block columns: 64 at a time in one VGPR (lane l: colind[k0 + 64c + l]), the next chunk in flight
  int ccur = 0, cnext = 0, cstamp = 0;
  auto load_cols = [&](int kstart) {
    const unsigned off = 4u * (unsigned)min(kstart + lane, k1 - 1);
    asm volatile("global_load_dword %0, %1, %2" : "=&v"(cnext) : "v"(off), "s"(colind) : "memory");
    cstamp = ++nis;
  };
  auto issue_a = [&](int kr) {  // blocks k0 + kr, k0 + kr + 1 (kr even) -> slots kr, kr + 1
    const int blk = (DIAG & 4) ? k0 : min(k0 + kr + h, k1 - 1);
    __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)blk * 256 + 8 * (lane & 31)),
                                     (lds_void_t)(smem + (kr & (NA - 1)) * 512), 16, 0, 0);
    ++nis;
  };
  if (k0 < k1) load_cols(k0);
  int ast[DA / 2 + 1];  // count at each A pair in flight
#pragma unroll
  for (int q = 0; q <= DA / 2; ++q) {
    if (k0 + 2 * q < k1) {
      issue_a(2 * q);
      ast[q] = nis;
    } else {
      ast[q] = -64;
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
      asm volatile(SPMM_VM_LADDER("%1") "v_mov_b32 %0, %2"
                   : "=&v"(ccur)
                   : "s"(nis - cstamp), "v"(cnext)
                   : "scc", "memory");
      if (k0 + kr + 64 < k1) load_cols(k0 + kr + 64);
    }
    const bool two = k0 + kr + 1 < k1;
    const int bc0 = __builtin_amdgcn_readlane(ccur, kr & 63);
    const int bc1 = __builtin_amdgcn_readlane(ccur, (kr + 1) & 63);
    wait_vm_older(nis - ast[0]);  // pair kr / 2 landed
#pragma unroll
    for (int q = 0; q < DA / 2; ++q) ast[q] = ast[q + 1];
    if (k0 + kr + DA + 2 < k1) {
      issue_a(kr + DA + 2);
      ast[DA / 2] = nis;
    } else {
      ast[DA / 2] = -64;
    }
    unsigned x[8];
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
    unsigned m[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned long long b =
          __builtin_amdgcn_ballot_w64(((x[4 * u] | x[4 * u + 1] | x[4 * u + 2] | x[4 * u + 3]) & 0x7fffu) != 0u);
      const unsigned w = (unsigned)b | (unsigned)(b >> 32);
      m[u] = (w | (w >> 16)) & 0xffffu;
    }
    if (!two) m[1] = 0u;  // the pair's second copy repeated the last block
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
      // consume the item issued P slots ago
      if (kind[s]) {
        wait_vm_older(nis - stamp[s]);
        f16x4 fb[kT];
        if constexpr (FLR) {
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
              : "v"(tra[0]), "v"(tra[1]), "v"(tra[2]), "v"(tra[3]), "v"(tra[4]), "v"(tra[5]),
                "v"(tra[6]), "v"(tra[7]), "n"(s * kStage)
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
                "v"(tra[14]), "v"(tra[15]), "n"(s * kStage)
              : "memory");
        } else if constexpr (FLC) {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %16\n\t"
              "ds_read_b64_tr_b16 %1, %16 offset:32\n\t"
              "ds_read_b64_tr_b16 %2, %16 offset:64\n\t"
              "ds_read_b64_tr_b16 %3, %16 offset:96\n\t"
              "ds_read_b64_tr_b16 %4, %16 offset:128\n\t"
              "ds_read_b64_tr_b16 %5, %16 offset:160\n\t"
              "ds_read_b64_tr_b16 %6, %16 offset:192\n\t"
              "ds_read_b64_tr_b16 %7, %16 offset:224\n\t"
              "ds_read_b64_tr_b16 %8, %16 offset:256\n\t"
              "ds_read_b64_tr_b16 %9, %16 offset:288\n\t"
              "ds_read_b64_tr_b16 %10, %16 offset:320\n\t"
              "ds_read_b64_tr_b16 %11, %16 offset:352\n\t"
              "ds_read_b64_tr_b16 %12, %16 offset:384\n\t"
              "ds_read_b64_tr_b16 %13, %16 offset:416\n\t"
              "ds_read_b64_tr_b16 %14, %16 offset:448\n\t"
              "ds_read_b64_tr_b16 %15, %16 offset:480\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7]), "=&v"(fb[8]), "=&v"(fb[9]),
                "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]), "=&v"(fb[13]), "=&v"(fb[14]),
                "=&v"(fb[15])
              : "v"(tro + (unsigned)(s * kStage))
              : "memory");
        } else if constexpr (COLS == 256) {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %16\n\t"
              "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %16 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %16 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %16 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %16 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %16 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %16 offset:3584\n\t"
              "ds_read_b64_tr_b16 %8, %16 offset:4096\n\t"
              "ds_read_b64_tr_b16 %9, %16 offset:4608\n\t"
              "ds_read_b64_tr_b16 %10, %16 offset:5120\n\t"
              "ds_read_b64_tr_b16 %11, %16 offset:5632\n\t"
              "ds_read_b64_tr_b16 %12, %16 offset:6144\n\t"
              "ds_read_b64_tr_b16 %13, %16 offset:6656\n\t"
              "ds_read_b64_tr_b16 %14, %16 offset:7168\n\t"
              "ds_read_b64_tr_b16 %15, %16 offset:7680\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7]), "=&v"(fb[8]), "=&v"(fb[9]),
                "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]), "=&v"(fb[13]), "=&v"(fb[14]),
                "=&v"(fb[15])
              : "v"(tro + (unsigned)(s * kStage))
              : "memory");
        } else {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %8\n\t"
              "ds_read_b64_tr_b16 %1, %8 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %8 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %8 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %8 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %8 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %8 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %8 offset:3584\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7])
              : "v"(tro + (unsigned)(s * kStage))
              : "memory");
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
          if (!(DIAG & 1)) acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa[s], fb[t], acc[t], 0, 0, 0);
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
          const char* base = r16 < cnt && !(DIAG & 2) ? reinterpret_cast<const char*>(B) + (size_t)r * ldb2 : zrow;
          char* const stage = smem + kStg + s * kStage;
          if constexpr (BUILD) {
            // record: 16 B-row indices (-1: padding), then the A fragment of lane L at 64 + 8 L
            char* const rec = items + (size_t)(k0 + nit) * kIsRec;
            // every lane stores (lanes 16-63 repeat lanes 0-15: no divergent branch)
            *reinterpret_cast<int*>(rec + 4 * r16) = r16 < cnt ? r : -1;
            unsigned ym0 = y[0], ym1 = y[1];
            if (cnt < 16) {
              const int e = 4 * g;
              ym0 &= (e < cnt ? 0xffffu : 0u) | (e + 1 < cnt ? 0xffff0000u : 0u);
              ym1 &= (e + 2 < cnt ? 0xffffu : 0u) | (e + 3 < cnt ? 0xffff0000u : 0u);
            }
            *reinterpret_cast<u32x2*>(rec + 64 + 8 * lane) = u32x2{ym0, ym1};
            nis += 2;
            ++nit;
            ebase = (ebase + 16) % CAP;
            npend = npend > 16 ? npend - 16 : 0;
            continue;
          }
          if constexpr (FLR) {
            int rw[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) rw[e] = __builtin_amdgcn_readlane(r, e);
            const bool hi = lane >= 32;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int e = 2 * j + (hi ? 1 : 0);
              const int re = hi ? rw[2 * j + 1] : rw[2 * j];
              const char* be = e < cnt && !(DIAG & 2) ? reinterpret_cast<const char*>(B) + (size_t)re * ldb2 : zrow;
              __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boffr[j]),
                                               (lds_void_t)(stage + 1024 * j), 16, 0, 0);
            }
            nis += 8;
          } else if constexpr (FLC) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int re = __builtin_amdgcn_readlane(r, e);
              const char* be = e < cnt ? reinterpret_cast<const char*>(B) + (size_t)re * ldb2 : zrow;
              __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boffl),
                                               (lds_void_t)(stage + kRowP * e), 4, 0, 0);
              __builtin_amdgcn_global_load_lds((gbl_void_t)(be + boffh),
                                               (lds_void_t)(stage + kRowP * e + 256), 4, 0, 0);
            }
            nis += 32;
          } else if constexpr (!(DIAG & 8)) {
#pragma unroll
            for (int j = 0; j < kCopies; ++j)
              __builtin_amdgcn_global_load_lds((gbl_void_t)(base + boff[j]),
                                               (lds_void_t)(stage + 1024 * j), 16, 0, 0);
            nis += kCopies;
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
  // nothing is in flight after the last round (a block-column chunk may be);
  // the full wait makes that visible to the register check (tests/test_isa_waits.py)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (BUILD) {
    if (lane == 0) nitems[br] = nit;
    return;
  }

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
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const int j = jt + 16 * t + r16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = C + row * ldc + j;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16, item stream (IS16; ROW blocks, row-major B): two launches.
// The column stream above walks each block row once per 256-column tile, and
// its chain A copy -> column mask -> push -> B-row copies runs at 7 waves per CU
// (22 KB of LDS each). Diagnostic builds of it (profiles/r02_cs16_diag.jsonl)
// put ~2.3 ms of its 4.5 in that walk: with no MFMA, no B rows and no item
// copies it still takes 2.27 ms. Here the walk runs ONCE per block row, as
// bsr16_f16_cs_kernel<BUILD> at ~24 waves per CU (6 KB of LDS: no item stage),
// and stores each item as a 576-B record: 16 B-row indices (-1: a padding
// entry, read from the zero row) and the MFMA A fragment of lane L at 64 + 8 L.
// Item records of block row br start at record rowptr[br] (a block row emits at
// most one item per block: a block adds at most 16 entries), nitems[br] counts them.
// This kernel then streams the records: one wave per (block row, COLS output
// columns), no dependence on A, so record r + R is in flight while item r's
// B rows are copied and item r - P + 1 is multiplied:
//  * record ring (R slots x 1 KB): one global_load_lds_dwordx4 per record
//    (lanes 36-63 repeat lane 35's 16 B: no divergent branch), issued R items ahead;
//  * item stage (P slots x 16 rows x COLS fp16): the copies of
//    bsr16_f16_cs_kernel (one ds_read_b32 of the record gives lane L the row of
//    entry L & 15), consumed P - 1 items later by 16 ds_read_b64_tr_b16 and 16
//    MFMAs, in the same item order and with the same fragments as the column
//    stream: the result is bit-identical to bsr16_f16_cs_kernel's.
// Every vector-memory operation of the loop is an LDS-DMA copy, counted in nis;
// waits are the run-time ladder (wait_vm_older), LDS reads inline asm ending in
// lgkmcnt(0), as in the column stream.
// ---------------------------------------------------------------------------
template <bool CROW, int P, int R, int COLS = 256>
__global__ __launch_bounds__(64) void bsr16_f16_is_kernel(
    int mb, int n, const int* __restrict__ rowptr, const char* __restrict__ items,
    const int* __restrict__ nitems, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, const int* __restrict__ order) {
  static_assert(P >= 2 && P <= 4 && R % P == 0 && R <= 8, "ring depths");
  static_assert(COLS == 128 || COLS == 256, "column tile");
  constexpr int kT = COLS / 16;
  constexpr int kCopies = COLS / 32;
  constexpr int kStage = 16 * COLS * 2;
  constexpr int kRecs = P * kStage;  // record ring after the item stages
  constexpr int kRecSlot = 1024;     // one record copy: 64 lanes x 16 B (lanes 36-63 repeat 35)
  constexpr int kLds = kRecs + R * kRecSlot;
  static_assert(kLds >= COLS * 16 * 4, "column-major C tile fits");
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int lane = threadIdx.x;
  const int g = lane >> 4, r16 = lane & 15;
  const int br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, 32);
  const int jt = blockIdx.y * COLS;
  const int k0 = rowptr[br], ni = nitems[br];
  const unsigned lds0 = lds_addr(smem);
  unsigned boff[kCopies];
#pragma unroll
  for (int j = 0; j < kCopies; ++j) boff[j] = 2u * (unsigned)min(jt + 8 * (4 * j + g), n - 8);
  const size_t ldb2 = (size_t)ldb * 2;
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 2 * (size_t)jt;
  const unsigned tro = lds0 + 256u * ((lane & 3) >> 1) + 16u * (4 * g + ((lane >> 2) & 3)) +
                       8u * (lane & 1);
  const char* const rec0 = items + (size_t)k0 * kIsRec + 16 * min(lane, 35);

  int nis = 0;
  int rstamp[R], stamp[P];
  f16x4 fa[P];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    rstamp[q] = -64;
    if (q < ni) {
      __builtin_amdgcn_global_load_lds((gbl_void_t)(rec0 + (size_t)q * kIsRec),
                                       (lds_void_t)(smem + kRecs + q * kRecSlot), 16, 0, 0);
      rstamp[q] = ++nis;
    }
  }
#pragma unroll
  for (int s = 0; s < P; ++s) {
    stamp[s] = -64;
    fa[s] = f16x4{0, 0, 0, 0};
  }
  f32x4 acc[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int i0 = 0; i0 < ni + P - 1; i0 += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int i = i0 + u;
      if (i < ni) {
        const int s = u % P;
        wait_vm_older(nis - rstamp[u]);  // record i landed
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        u32x2 y;
        int r;
        asm volatile("ds_read_b32 %0, %2\n\t"
                     "ds_read_b64 %1, %3\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(r), "=&v"(y)
                     : "v"(lds0 + kRecs + u * kRecSlot + 4u * r16),
                       "v"(lds0 + kRecs + u * kRecSlot + 64u + 8u * lane)
                     : "memory");
        const char* base = r >= 0 ? reinterpret_cast<const char*>(B) + (size_t)r * ldb2 : zrow;
        char* const stage = smem + s * kStage;
#pragma unroll
        for (int j = 0; j < kCopies; ++j)
          __builtin_amdgcn_global_load_lds((gbl_void_t)(base + boff[j]),
                                           (lds_void_t)(stage + 1024 * j), 16, 0, 0);
        nis += kCopies;
        stamp[s] = nis;
        const unsigned uy[2] = {y[0], y[1]};
        fa[s] = *reinterpret_cast<const f16x4*>(uy);
        // the slot just read takes record i + R
        if (i + R < ni) {
          __builtin_amdgcn_global_load_lds((gbl_void_t)(rec0 + (size_t)(i + R) * kIsRec),
                                           (lds_void_t)(smem + kRecs + u * kRecSlot), 16, 0, 0);
          rstamp[u] = ++nis;
        }
      }
      const int j = i - P + 1;
      if (j >= 0 && j < ni) {
        const int s = (u + 1) % P;  // j % P (i0 is a multiple of R, R of P)
        wait_vm_older(nis - stamp[s]);
        f16x4 fb[kT];
        if constexpr (COLS == 256) {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %16\n\t"
              "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %16 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %16 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %16 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %16 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %16 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %16 offset:3584\n\t"
              "ds_read_b64_tr_b16 %8, %16 offset:4096\n\t"
              "ds_read_b64_tr_b16 %9, %16 offset:4608\n\t"
              "ds_read_b64_tr_b16 %10, %16 offset:5120\n\t"
              "ds_read_b64_tr_b16 %11, %16 offset:5632\n\t"
              "ds_read_b64_tr_b16 %12, %16 offset:6144\n\t"
              "ds_read_b64_tr_b16 %13, %16 offset:6656\n\t"
              "ds_read_b64_tr_b16 %14, %16 offset:7168\n\t"
              "ds_read_b64_tr_b16 %15, %16 offset:7680\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7]), "=&v"(fb[8]), "=&v"(fb[9]),
                "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]), "=&v"(fb[13]), "=&v"(fb[14]),
                "=&v"(fb[15])
              : "v"(tro + (unsigned)(s * kStage))
              : "memory");
        } else {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %8\n\t"
              "ds_read_b64_tr_b16 %1, %8 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %8 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %8 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %8 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %8 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %8 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %8 offset:3584\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7])
              : "v"(tro + (unsigned)(s * kStage))
              : "memory");
        }
#pragma unroll
        for (int t = 0; t < kT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa[s], fb[t], acc[t], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  if constexpr (!CROW) {
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
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const int j = jt + 16 * t + r16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = C + row * ldc + j;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16, item stream with register-staged B rows (IS16R; the second
// launch after the same builder). The kernel trace of bsr16_f16_is_kernel shows
// the walk is not what bounds the column stream: without it the streaming
// kernel alone takes 4.43 ms against 4.51 for the whole column stream, and the
// builder 0.76 ms (profiles/r02_is16_kt). What bounds both is the B bytes in
// flight: the LDS item stages hold them, and 5-8 waves per CU with 1-2 stages
// in flight each keep ~80 KB per CU outstanding. Here the B rows of the next D
// items travel in VGPRs (32 per item and lane: lane L holds, for copy j, row
// L & 15, 16-B chunk 4j + L / 16, the LDS-DMA layout of the column stream) and
// only the item being multiplied passes through LDS (8 ds_write_b128 into the
// same chunk-major stage, then the same 16 ds_read_b64_tr_b16): D x 8 KB per
// wave in flight at one 8-KB stage of LDS. Records and B rows are plain loads
// (the compiler's own vmcnt waits); the stage's writes and reads are one
// wave's, in LDS order. Same items, same order, same fragments: bit-identical
// to bsr16_f16_cs_kernel.
// ---------------------------------------------------------------------------
template <bool CROW, int D, int COLS = 256, bool FL = false>
__global__ __launch_bounds__(64) void bsr16_f16_isr_kernel(
    int mb, int n, const int* __restrict__ rowptr, const char* __restrict__ items,
    const int* __restrict__ nitems, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, const int* __restrict__ order) {
  static_assert(D >= 1 && D <= 4, "items in flight");
  static_assert(COLS == 128 || COLS == 256, "column tile");
  static_assert(!FL || COLS == 256, "full-line loads: 256 columns");
  constexpr int DR = 2 * D;  // records in flight (the next D items' rows are needed D early)
  constexpr int kT = COLS / 16;
  constexpr int kCopies = COLS / 32;
  // FL: chunk stride 272 B (16 rows x 16 B + 16): row j of chunk c at bank slot c + j, so the
  // 8-B writes of one row (chunks 0-31) and the transposed reads (16 rows of one chunk) are
  // conflict-free, and chunk 2t + 1 stays an immediate offset (544 t) from chunk 2t
  constexpr int kCs = FL ? 272 : 256;
  constexpr int kStage = FL ? 32 * kCs : 16 * COLS * 2;
  constexpr int kLds = CROW ? kStage : (kStage > COLS * 64 ? kStage : COLS * 64);
  constexpr int kLoads = FL ? 16 : kCopies;  // B loads per item and lane
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x;
  const int g = lane >> 4, r16 = lane & 15;
  const int br = order ? order[blockIdx.x] : xcd_block_row(blockIdx.x, mb, 32);
  const int jt = blockIdx.y * COLS;
  const int k0 = rowptr[br], ni = nitems[br];
  const unsigned lds0 = lds_addr(smem);
  unsigned boff[kCopies];
#pragma unroll
  for (int j = 0; j < kCopies; ++j) boff[j] = 2u * (unsigned)min(jt + 8 * (4 * j + g), n - 8);
  const size_t ldb2 = (size_t)ldb * 2;
  const char* const zrow = reinterpret_cast<const char*>(g_zero_row) - 2 * (size_t)jt;
  const unsigned tro = lds0 + (unsigned)kCs * ((lane & 3) >> 1) + 16u * (4 * g + ((lane >> 2) & 3)) +
                       8u * (lane & 1);
  // FL: lane L loads 8 B (columns 4L .. 4L + 3) of one B row per load, 16 loads per item
  const unsigned boffl = 2u * (unsigned)min(jt + 4 * lane, n - 4);
  char* const wfl = smem + kCs * (lane >> 1) + 8 * (lane & 1);
  const char* const recs = items + (size_t)k0 * kIsRec;

  f32x4 acc[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int rrow[DR];
  u32x2 ra[DR];
  typedef typename std::conditional<FL, u32x2, u32x4>::type bvec;
  bvec bq[D][kLoads];
  // Every load is issued whatever the item count (records clamped to the last
  // one, B rows of items past the end from the zero row): with loads under
  // branches hipcc's waits merge pessimistically and wait for every
  // outstanding load before each item (vmcnt(0)); straight-line issue keeps
  // its counts exact, so item i waits only for its own rows.
  auto load_rec = [&](int q, int i) {
    const char* rec = recs + (size_t)min(i, ni - 1) * kIsRec;
    rrow[q] = *reinterpret_cast<const int*>(rec + 4 * r16);
    ra[q] = *reinterpret_cast<const u32x2*>(rec + 64 + 8 * lane);
  };
  auto load_b = [&](int d, int q, bool live) {
    if constexpr (FL) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int rj = __builtin_amdgcn_readlane(rrow[q], j);
        const char* base = live && rj >= 0 ? reinterpret_cast<const char*>(B) + (size_t)rj * ldb2 : zrow;
        bq[d][j] = *reinterpret_cast<const bvec*>(base + boffl);
      }
    } else {
      const char* base = live && rrow[q] >= 0 ? reinterpret_cast<const char*>(B) + (size_t)rrow[q] * ldb2 : zrow;
#pragma unroll
      for (int j = 0; j < kCopies; ++j) bq[d][j] = *reinterpret_cast<const bvec*>(base + boff[j]);
    }
  };
  if (ni > 0) {
#pragma unroll
    for (int q = 0; q < DR; ++q) load_rec(q, q);
#pragma unroll
    for (int d = 0; d < D; ++d) load_b(d, d, d < ni);
  }

  for (int i0 = 0; i0 < ni; i0 += DR) {
#pragma unroll
    for (int u = 0; u < DR; ++u) {
      const int i = i0 + u;
      if (i < ni) {
        const int d = u % D;  // i % D (i0 is a multiple of DR, DR of D)
        // item i: its rows to the stage, transposed reads, MFMAs
        if constexpr (FL) {
#pragma unroll
          for (int j = 0; j < 16; ++j) *reinterpret_cast<bvec*>(wfl + 16 * j) = bq[d][j];
        } else {
#pragma unroll
          for (int j = 0; j < kCopies; ++j)
            *reinterpret_cast<bvec*>(smem + 1024 * j + 16 * lane) = bq[d][j];
        }
        f16x4 fb[kT];
        if constexpr (FL) {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %16\n\t"
              "ds_read_b64_tr_b16 %1, %16 offset:544\n\t"
              "ds_read_b64_tr_b16 %2, %16 offset:1088\n\t"
              "ds_read_b64_tr_b16 %3, %16 offset:1632\n\t"
              "ds_read_b64_tr_b16 %4, %16 offset:2176\n\t"
              "ds_read_b64_tr_b16 %5, %16 offset:2720\n\t"
              "ds_read_b64_tr_b16 %6, %16 offset:3264\n\t"
              "ds_read_b64_tr_b16 %7, %16 offset:3808\n\t"
              "ds_read_b64_tr_b16 %8, %16 offset:4352\n\t"
              "ds_read_b64_tr_b16 %9, %16 offset:4896\n\t"
              "ds_read_b64_tr_b16 %10, %16 offset:5440\n\t"
              "ds_read_b64_tr_b16 %11, %16 offset:5984\n\t"
              "ds_read_b64_tr_b16 %12, %16 offset:6528\n\t"
              "ds_read_b64_tr_b16 %13, %16 offset:7072\n\t"
              "ds_read_b64_tr_b16 %14, %16 offset:7616\n\t"
              "ds_read_b64_tr_b16 %15, %16 offset:8160\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7]), "=&v"(fb[8]), "=&v"(fb[9]),
                "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]), "=&v"(fb[13]), "=&v"(fb[14]),
                "=&v"(fb[15])
              : "v"(tro)
              : "memory");
        } else if constexpr (COLS == 256) {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %16\n\t"
              "ds_read_b64_tr_b16 %1, %16 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %16 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %16 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %16 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %16 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %16 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %16 offset:3584\n\t"
              "ds_read_b64_tr_b16 %8, %16 offset:4096\n\t"
              "ds_read_b64_tr_b16 %9, %16 offset:4608\n\t"
              "ds_read_b64_tr_b16 %10, %16 offset:5120\n\t"
              "ds_read_b64_tr_b16 %11, %16 offset:5632\n\t"
              "ds_read_b64_tr_b16 %12, %16 offset:6144\n\t"
              "ds_read_b64_tr_b16 %13, %16 offset:6656\n\t"
              "ds_read_b64_tr_b16 %14, %16 offset:7168\n\t"
              "ds_read_b64_tr_b16 %15, %16 offset:7680\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7]), "=&v"(fb[8]), "=&v"(fb[9]),
                "=&v"(fb[10]), "=&v"(fb[11]), "=&v"(fb[12]), "=&v"(fb[13]), "=&v"(fb[14]),
                "=&v"(fb[15])
              : "v"(tro)
              : "memory");
        } else {
          asm volatile(
              "ds_read_b64_tr_b16 %0, %8\n\t"
              "ds_read_b64_tr_b16 %1, %8 offset:512\n\t"
              "ds_read_b64_tr_b16 %2, %8 offset:1024\n\t"
              "ds_read_b64_tr_b16 %3, %8 offset:1536\n\t"
              "ds_read_b64_tr_b16 %4, %8 offset:2048\n\t"
              "ds_read_b64_tr_b16 %5, %8 offset:2560\n\t"
              "ds_read_b64_tr_b16 %6, %8 offset:3072\n\t"
              "ds_read_b64_tr_b16 %7, %8 offset:3584\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]), "=&v"(fb[4]),
                "=&v"(fb[5]), "=&v"(fb[6]), "=&v"(fb[7])
              : "v"(tro)
              : "memory");
        }
        const u32x2 a2 = ra[u];
        const unsigned uy[2] = {a2[0], a2[1]};
        const f16x4 fa = *reinterpret_cast<const f16x4*>(uy);
#pragma unroll
        for (int t = 0; t < kT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa, fb[t], acc[t], 0, 0, 0);
      }
      // item i + D's rows into the registers just freed (its record is q = (u + D) % DR),
      // then record i + DR into record slot u
      load_b(u % D, (u + D) % DR, i + D < ni);
      load_rec(u, i + DR);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight at the epilogue

  if constexpr (!CROW) {
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
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const int j = jt + 16 * t + r16;
    if (j >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t row = (size_t)br * 16 + 4 * g + e;
      float* p = C + row * ldc + j;
      *p = epi(acc[t][e], alpha, beta, p);
    }
  }
}

// ---------------------------------------------------------------------------
// bs = 16 fp16, LDS-staged, TWO block rows per workgroup sharing B panels:
// the workgroup walks the union of the two rows' block columns, copying each
// B panel once (products stand-in: the union is 0.73 of the two rows' blocks).
// Waves 0 / 1 copy the A block of row 0 / 1, all four copy a quarter of the
// panel; the union element's row mask reaches the compute step through an
// LDS header per stage. Past the end, "end" headers and dummy copies keep
// every iteration's copy count fixed (counted vmcnt per wave).
// ---------------------------------------------------------------------------
template <bool CROW, int D>
__global__ __launch_bounds__(256) void bsr16_f16_pair_kernel(
    int mb, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const _Float16* __restrict__ val, const _Float16* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc) {
  typedef _Float16 T;
  constexpr int kEpc = 8, kA = 512, kRowB = 512, kStage = 2 * 1024 + 16 * kRowB;
  __shared__ __attribute__((aligned(16))) char smem[D * kStage];
  __shared__ int hdr[D];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int ng = (mb + 1) / 2;
  int grp = blockIdx.x;
  {  // XCD-contiguous groups
    const int q = ng / 8, rem = ng % 8, x = grp % 8, i = grp / 8;
    grp = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + i;
  }
  const int br0 = 2 * grp;
  const int jt = blockIdx.y * 256;
  const int g = lane >> 4, c16 = lane & 15;
  int pos[2], end[2], head[2];
  bool any = false;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int br = br0 + q;
    pos[q] = br < mb ? rowptr[br] : 0;
    end[q] = br < mb ? rowptr[br + 1] : 0;
    any |= pos[q] < end[q];
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[q][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (any) {
    ColCursor c0(colind, pos[0], end[0], lane), c1(colind, pos[1], end[1], lane);
    head[0] = pos[0] < end[0] ? c0.get(pos[0]) : INT_MAX;
    head[1] = pos[1] < end[1] ? c1.get(pos[1]) : INT_MAX;
    const int safe_k = pos[0] < end[0] ? pos[0] : pos[1];
    const int a_off = (lane * 16 % kA) / 2;  // lanes 32-63 duplicate lanes 0-31
    int b_src[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 4 * wv + 2 * i + lane / 32;
      const int c = (lane % 32) ^ bsr16_swz<T>(row);
      b_src[i] = row * ldb + min(jt + c * kEpc, n - kEpc);
    }
    auto issue_next = [&](int st) {
      const int c = min(head[0], head[1]);
      int mask = 0, k0i = pos[0] < end[0] ? pos[0] : safe_k, k1i = pos[1] < end[1] ? pos[1] : safe_k;
      if (c != INT_MAX && head[0] == c) {
        mask |= 1;
        ++pos[0];
        head[0] = pos[0] < end[0] ? c0.get(pos[0]) : INT_MAX;
      }
      if (c != INT_MAX && head[1] == c) {
        mask |= 2;
        ++pos[1];
        head[1] = pos[1] < end[1] ? c1.get(pos[1]) : INT_MAX;
      }
      char* stage = smem + st * kStage;
      if (threadIdx.x == 0) hdr[st] = c == INT_MAX ? -1 : mask;
      if (wv < 2)
        __builtin_amdgcn_global_load_lds((gbl_void_t)(val + (size_t)(wv ? k1i : k0i) * 256 + a_off),
                                         (lds_void_t)(stage + wv * 1024), 16, 0, 0);
      const T* bp = B + (size_t)(c == INT_MAX ? 0 : c) * 16 * ldb;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((gbl_void_t)(bp + b_src[i]),
                                         (lds_void_t)(stage + 2048 + (4 * wv + 2 * i) * kRowB),
                                         16, 0, 0);
    };
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issue_next(d);
    int st = 0;
    while (true) {
      if (wv < 2)
        __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(3 * (D - 2)));
      else
        __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(2 * (D - 2)));
      __builtin_amdgcn_s_barrier();
      const int mask = __builtin_amdgcn_readfirstlane(hdr[st]);
      if (mask < 0) break;
      issue_next(st == 0 ? D - 1 : st - 1);
      const char* stage = smem + st * kStage;
      const char* bpan = stage + 2048;
      const int q4 = (lane >> 2) & 3, p4 = lane & 3;
      const int row = 4 * g + q4;
      f16x4 fb[4];
      unsigned ad[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = 64 * wv + 16 * t + 4 * p4;
        ad[t] = lds_addr(bpan + row * kRowB + (((col >> 3) ^ bsr16_swz<T>(row)) << 4) + (col & 7) * 2);
      }
      ds_read_tr16_n(fb, ad);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (!((mask >> q) & 1)) continue;
        const f16x4 fa = ds_read_f16x4(lds_addr(stage + q * 1024 + c16 * 32 + 8 * g));
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[q][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(fa, fb[t], acc[q][t], 0, 0, 0);
      }
      st = st == D - 1 ? 0 : st + 1;
    }
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int br = br0 + q;
    if (br >= mb) break;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = jt + 64 * wv + 16 * t + c16;
      if (j >= n) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t r = (size_t)br * 16 + 4 * g + e;
        float* p = CROW ? C + r * ldc + j : C + (size_t)j * ldc + r;
        *p = epi(acc[q][t][e], alpha, beta, p);
      }
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

constexpr int kBsr32Default = 40;
// LDS-staged bs = 32 kernel: 4096 + D (+ 8: XCD-contiguous order; 4123-4125:
// XCD order in chunks of 16 / 32 / 64 block rows). 42 D DA: column-masked,
// B stages D, A stages DA; (2, 5) fits 3 workgroups per CU and is the
// fastest measured (reddit stand-in 2.65 ms vs 4.57 for 4124; products bs = 32
// 4.62 vs 8.51; (3, 6) 3.08 / 5.60; (4, 8) 4.87 / 9.09).
// Column stream with register items (bsr32_f32_cs2_kernel, 6 item slots, 3 A
// slots): products stand-in 3.05 ms, reddit 2.01 (4583, the LDS item ring:
// 3.21 / 2.16; CM4 4402: 4.38 / 2.59; profiles/r02_cs_sweep.jsonl,
// r02_cs2_sweep.jsonl). With 32-bit row offsets in the B loads (4556, O32):
// products 3.02 vs 3.11, reddit 2.04 vs 2.05 (profiles/r02_bsr_order_sweep.jsonl);
// 4596 where 32 * ldb * 4 does not fit 31 bits. With cross-block pairs (4516,
// PK): reddit 2.01-2.02 vs 2.04-2.05, products 3.31 vs 3.30 (same box,
// profiles/r02_cs2_pk_sweep.jsonl).
constexpr int kBsr32LdsDefault = 4516;
constexpr int kBsr32LdsDefaultWideLdb = 4596;
// Blocks known to be dense (the hybrid's BSR part, MFMA-pipe bound): the
// full-panel kernel with D = 2 (40 KB, 4 workgroups per CU) and the chunked
// XCD order. Products stand-in hybrid part 1.71 vs 1.87 ms for D = 3 (4124),
// 1.90 for D = 4; reddit 0.85 vs 0.86.
constexpr int kBsr32LdsDense = 4126;
// LDS-staged bs = 16 kernels: 4096 + D (+ 8: XCD-contiguous block rows). fp16:
// 6 waves/SIMD at D = 3 beat deeper rings, the XCD order 5 % more
// (products_bsr16_f16 8.80 ms vs 10.38 for the register-fragment kernel);
// fp32: D = 4, 18.4 vs 21.4.
// 46 D DA: column-masked bs = 16 (bsr16_cm_kernel), B stages D, A stages DA.
// products stand-in bs = 16 K = 512: fp16 (2, 5) 7.41 ms vs 8.81 for the
// block-row pair kernel 4303, (3, 6) 9.40; fp32 (2, 5) 16.6 vs 18.5 for 4100.
// 47 D DA: the same with amdgpu_waves_per_eu(8) (52 VGPRs, no AGPRs: 8 waves
// per SIMD instead of 7): fp16 7.19 ms.
constexpr int kBsr16LdsDefault = 4625;
constexpr int kBsr16F16LdsDefault = 4725;
// 48 D DA: 512 output columns per workgroup (A once per 512 columns, 8 tiles
// per wave): products stand-in K = 512 6.89 ms vs 7.08 for 4725.
constexpr int kBsr16F16LdsWide = 4825;
// Column stream (bsr16_f16_cs_kernel, 2 item stages, NA = 8, DA = 4): products
// stand-in K = 512 4.57 ms vs 5.94 for 4825 (profiles/r02_cs16_v3_sweep.jsonl);
// with two whole B rows per 16-B copy (FLR, 6121): 4.09 vs 4.48-4.49 for 5021 on
// the same box, bit-identical (profiles/r02_is16/sweeps.txt); with the 48-entry
// pending list and a 4-slot A ring (6104: 19.7 KB, 8 waves per CU instead of 7)
// 4.04 vs 4.18-4.19 for 6121 on one box.
constexpr int kBsr16F16Cs = 6104;
constexpr int kBsr16Default = 8;     // fp32 bs 16
constexpr int kBsr16F16Default = 12;  // fp16 bs 16

// SPMM_BSR_VARIANT=<v> overrides the variant of the row/row/row launch of
// the bs 32 and bs 16 kernels (tuning sweeps only; tools/bsr_variants.sh).
int variant_override() {
  static const int var = [] {
    const char* e = getenv("SPMM_BSR_VARIANT");
    return e ? atoi(e) : -1;
  }();
  return var;
}
#define SPMM_COMMA ,

// Block-row order for the column-stream kernels: longest first when the grid
// is at most kLptRounds waves per resident slot deep (a few long rows would
// otherwise start last and run alone), else nullptr (the kernels' XCD-chunked
// order, which keeps neighbouring block rows in one L2). SPMM_BSR_ORDER=1
// forces longest first, 2 the XCD order (tuning). One launch of
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
  static const int force = [] {
    const char* e = getenv("SPMM_BSR_ORDER");
    return e ? atoi(e) : 0;
  }();
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
                              int m = 0) {
  static const int force = [] {
    const char* e = getenv("SPMM_BSR_ORDER");
    return e ? atoi(e) : 0;
  }();
  *order = nullptr;
  const long waves = (long)mb * ntiles, slots = slots_per_cu * ctx->num_cus;
  if (force == 2 || (force != 1 && force != 3 && waves > kLptRounds * slots))
    return SPMM_STATUS_SUCCESS;
  if (spmm_status_t st = spmm::ensure_order_buffer(ctx, mb)) return st;
  hipLaunchKernelGGL(block_row_order_kernel, dim3(1), dim3(1024), 0, ctx->stream, mb, rowptr,
                     crp, m, ctx->order);
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

spmm_status_t launch_bsrmm_f32(spmm_context* ctx, spmm_direction_t dir, int mb, int kb, int n,
                               int nnzb, int bs, float alpha, const int* rowptr,
                               const int* colind, const float* val, const float* B, int ldb,
                               spmm_order_t orderB, float beta, float* C, int ldc,
                               spmm_order_t orderC, bool dense_blocks) {
  (void)kb;
  if (mb == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const bool rowd = dir == SPMM_DIRECTION_ROW;
  const bool brow = orderB == SPMM_ORDER_ROW;
  const bool crow = orderC == SPMM_ORDER_ROW;
  const bool vec_ok = aligned(val, 16) && (brow || (aligned(B, 16) && ldb % 4 == 0));
  const int slot = timing_begin(ctx);
  const int var = variant_override();
  if (bs == 32 && rowd && brow && n >= 4 && n % 4 == 0 && ldb % 4 == 0 && aligned(val, 16) &&
      aligned(B, 16) && (var < 0 || var >= 4096)) {
    dim3 grid(mb, (n + 127) / 128);
    // 46xx / 47xx select bs = 16 kernels: the bs = 32 default here. Blocks known to
    // be dense (the hybrid's BSR part) take the full-panel kernel: with most
    // columns set the mask buys nothing and its deeper B ring wins (reddit
    // stand-in hybrid: 0.81 vs 0.96 ms).
    int lv = var < 0 || ((var % 1000) / 100 >= 6 && (var % 1000) / 100 <= 8) || var / 100 == 50 ||
                     var / 100 == 51 || var / 100 == 53 || var / 100 == 97 || (var / 100 >= 55 && var / 100 <= 61) ||
                     var / 100 == 63
                 ? (dense_blocks ? kBsr32LdsDense
                                 : ((size_t)ldb * 128 < (1u << 31) ? kBsr32LdsDefault
                                                                     : kBsr32LdsDefaultWideLdb))
                 : var;
    if ((lv == 4556 || lv == 4558 || lv == 4554 || lv == 4516 || lv == 4518 || lv == 4416) &&
        (size_t)ldb * 128 >= (1u << 31))
      lv = kBsr32LdsDefaultWideLdb;  // O32 needs 32-row panels addressable in 31 bits
#define L(D, X)                                                                                   \
  if (crow) hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, D, X>), grid, dim3(256), 0, ctx->stream,  \
                               mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, nullptr,  \
                               nullptr, nullptr, 0, nullptr);                                        \
  else hipLaunchKernelGGL((bsr32_f32_lds_kernel<false, D, X>), grid, dim3(256), 0, ctx->stream,      \
                          mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, nullptr,       \
                          nullptr, nullptr, 0, nullptr);
    // split-bf16 (opt-in): wave-pair split-K form for row-major C (products
    // hybrid 1.86-1.87 vs 1.89 ms fused, reddit 0.80 vs 0.83, profiles/r01_hybrid_split.jsonl), else one k range per wave
    if (dense_blocks && var < 0 && (ctx->hybrid_flags & SPMM_HYBRID_SPLIT_BF16))
      lv = crow ? 4927 : 4926;
    switch (lv) {
      case 4926:  // kBsr32LdsDense with split-bf16 products (SPMM_HYBRID_SPLIT_BF16)
        if (crow) hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, false, 24, true>), grid,
                                     dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,
                                     alpha, beta, C, ldc, nullptr, nullptr, nullptr, 0, nullptr);
        else hipLaunchKernelGGL((bsr32_f32_lds_kernel<false, 2, 32, false, 24, true>), grid,
                                dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb,
                                alpha, beta, C, ldc, nullptr, nullptr, nullptr, 0, nullptr);
        break;
      case 4927:  // 4926 with split-K over wave pairs (PAIR)
        if (!crow) { timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE; }
        hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, false, 24, true, true>), grid,
                           dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha,
                           beta, C, ldc, nullptr, nullptr, nullptr, 0, nullptr);
        break;
      case 4098: L(2, 0) break;
      case 4099: L(3, 0) break;
      case 4100: L(4, 0) break;
      case 4106: L(2, 1) break;
      case 4107: L(3, 1) break;
      case 4123: L(3, 16) break;  // 4123-4125: XCD order in chunks of 16 / 32 / 64
      case 4124: L(3, 32) break;
      case 4125: L(3, 64) break;
      case 4126: L(2, 32) break;  // D = 2 / 4 with the chunked XCD order
      case 4127: L(4, 32) break;
      // column-masked (fetch only the B rows of nonzero A columns): 42DA:
      // D = B stages, A = A stages (42 3 6 = D 3, DA 6); + 1000 = no MFMA (diagnostic)
#define CM(V, ...)                                                                                     \
  case V:                                                                                              \
    if (crow) hipLaunchKernelGGL((bsr32_f32_cm_kernel<true, 32, __VA_ARGS__>), grid, dim3(256), 0,      \
                                 ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
    else hipLaunchKernelGGL((bsr32_f32_cm_kernel<false, 32, __VA_ARGS__>), grid, dim3(256), 0,          \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);      \
    break;
      CM(4200, 3, 6) CM(4236, 3, 6) CM(4235, 3, 5) CM(4237, 3, 7) CM(4225, 2, 5) CM(4226, 2, 6)
      CM(4247, 4, 7) CM(4248, 4, 8) CM(5236, 3, 6, 1) CM(5225, 2, 5, 1)
      // diagnostics: 602x = D 2, DA 5 with DIAG x (1 no MFMA, 2 no B, 4 A from k0)
      CM(6022, 2, 5, 2) CM(6024, 2, 5, 4) CM(6026, 2, 5, 6) CM(6027, 2, 5, 7)
#undef CM
      // column stream (bsr32_f32_cs_kernel): 45PA = P item slots, NA A slots
#define CS(V, P, A)                                                                              \
  case V:                                                                                        \
    if (crow) hipLaunchKernelGGL((bsr32_f32_cs_kernel<true, 32, P, A>), grid, dim3(64), 0,       \
                                 ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, \
                                 ldc);                                                           \
    else hipLaunchKernelGGL((bsr32_f32_cs_kernel<false, 32, P, A>), grid, dim3(64), 0,           \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
    break;
      CS(4583, 8, 3) CS(4584, 8, 4) CS(4582, 8, 2) CS(4563, 6, 3) CS(4543, 4, 3) CS(4542, 4, 2)
      CS(4573, 7, 3) CS(4574, 7, 4)
#undef CS
      // column stream with register items (bsr32_f32_cs2_kernel): 459x =
      // (P, NA): 4593 (8, 3), 4594 (8, 4), 4592 (8, 2), 4596 (6, 3),
      // 4597 (4, 3), 4598 (12, 3), 4599 (16, 3)
#define CS2(V, P, A, ...)                                                                        \
  case V: {                                                                                      \
    const int* ord = nullptr;                                                                    \
    const int4 *sg = nullptr, *spl = nullptr;                                                    \
    float* pt = nullptr;                                                                         \
    int nsg = 0, nspl = 0;                                                                       \
    spmm_status_t st = SPMM_STATUS_SUCCESS;                                                      \
    if (crow) st = cs2_segments(ctx, mb, nnzb, grid.y, rowptr, &sg, &spl, &pt, &nsg, &nspl);     \
    if (st == SPMM_STATUS_SUCCESS && !sg) st = block_row_order(ctx, mb, grid.y, rowptr, &ord);   \
    if (st != SPMM_STATUS_SUCCESS) {                                                             \
      timing_end(ctx, slot);                                                                     \
      return st;                                                                                 \
    }                                                                                            \
    if (crow) {                                                                                  \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<true, 32, P, A, ##__VA_ARGS__>),                  \
                         dim3(sg ? nsg : mb, grid.y), dim3(64), 0, ctx->stream, mb, n, rowptr,    \
                         colind, val, B, ldb, alpha, beta, C, ldc, ord, sg, pt);                 \
      if (spl)                                                                                   \
        hipLaunchKernelGGL(seg_fixup_kernel, dim3(nspl, grid.y), dim3(256), 0, ctx->stream, n,   \
                           spl, pt, alpha, beta, C, ldc);                                        \
    } else {                                                                                     \
      hipLaunchKernelGGL((bsr32_f32_cs2_kernel<false, 32, P, A, ##__VA_ARGS__>), grid, dim3(64), \
                         0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, \
                         ord, nullptr, nullptr);                                                 \
    }                                                                                            \
    break;                                                                                       \
  }
      CS2(4593, 8, 3) CS2(4594, 8, 4) CS2(4592, 8, 2) CS2(4596, 6, 3) CS2(4597, 4, 3)
      CS2(4598, 12, 3) CS2(4599, 16, 3)
      // 455P: 32-bit row offsets in the load's VGPR offset (O32), P item slots, NA = 3
      CS2(4556, 6, 3, 0, true) CS2(4558, 8, 3, 0, true) CS2(4554, 4, 3, 0, true)
      // 457P... taken by CS; 4516 / 4518: O32 + cross-block pairs (PK), P = 6 / 8
      CS2(4516, 6, 3, 0, true, true) CS2(4518, 8, 3, 0, true, true)
      // 4416: 4516 with the A copies non-temporal (nt: A is read once, keep L2 for B rows)
      CS2(4416, 6, 3, 0, true, true, true)
      // diagnostics (wrong results): 960D = (6, 3) with DIAG D
      CS2(9601, 6, 3, 1) CS2(9602, 6, 3, 2) CS2(9604, 6, 3, 4) CS2(9606, 6, 3, 6)
      CS2(9607, 6, 3, 7)
#undef CS2
      case 4402:  // CM4: 4 workgroups per CU (bsr32_f32_cm4_kernel)
        if (crow) hipLaunchKernelGGL((bsr32_f32_cm4_kernel<true, 32>), grid, dim3(256), 0, ctx->stream,
                                     mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        else hipLaunchKernelGGL((bsr32_f32_cm4_kernel<false, 32>), grid, dim3(256), 0, ctx->stream,
                                mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        break;
      default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
    }
#undef L
  } else if (bs == 32 && vec_ok) {
    const int waves = n <= 32 ? 1 : (n <= 64 ? 2 : 4);
    dim3 grid(mb, (n + 32 * waves - 1) / (32 * waves));
    if (var >= 0 && var < 4096 && rowd && brow && crow) {
      switch (var) {
#define V(x) case x: hipLaunchKernelGGL((bsr32_f32_mfma_kernel<true, true, true, x>), grid, dim3(64 * waves), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); break;
        V(40) V(44) V(42) V(50) V(58) V(66) V(41) V(49)
#undef V
        default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
      }
    } else {
      SPMM_BSR_DISPATCH(bsr32_f32_mfma_kernel, SPMM_COMMA kBsr32Default, grid, dim3(64 * waves), ctx->stream, rowd, brow,
                        crow, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    }
  } else if (bs == 16 && rowd && brow && n >= 4 && n % 4 == 0 && ldb % 4 == 0 &&
             aligned(val, 16) && aligned(B, 16) && (var < 0 || var >= 4096)) {
    dim3 grid(mb, (n + 255) / 256);
    // 42xx / 52xx select bs = 32 kernels: the bs = 16 default here
    const int lv = var < 0 || (var % 1000) / 100 == 2 || var / 100 == 44 || var / 100 == 45 ||
                           var / 100 == 50 || var / 100 == 51 || var / 100 == 53 ||
                           var / 100 == 97 || (var / 100 >= 55 && var / 100 <= 61) || var / 100 == 63
                       ? kBsr16LdsDefault
                       : var;
#define L(D)                                                                                     \
  if (crow) hipLaunchKernelGGL((bsr16_lds_kernel<float, true, D>), grid, dim3(256), 0, ctx->stream, \
                               mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);         \
  else hipLaunchKernelGGL((bsr16_lds_kernel<float, false, D>), grid, dim3(256), 0, ctx->stream,     \
                          mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    switch (lv) {
      case 4099: L(3) break;
      case 4100: L(4) break;
      case 4102: L(6) break;
#define CM(V, ...)                                                                                  \
  case V:                                                                                           \
    if (crow) hipLaunchKernelGGL((bsr16_cm_kernel<float, true, __VA_ARGS__>), grid, dim3(256), 0,    \
                                 ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
    else hipLaunchKernelGGL((bsr16_cm_kernel<float, false, __VA_ARGS__>), grid, dim3(256), 0,        \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);   \
    break;
      CM(4625, 2, 5) CM(4636, 3, 6) CM(4626, 2, 6) CM(4646, 4, 6)  // column-masked, 46 D DA
#undef CM
      case 4108:  // + 8: XCD-contiguous block rows
        if (crow) hipLaunchKernelGGL((bsr16_lds_kernel<float, true, 4, true>), grid, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        else hipLaunchKernelGGL((bsr16_lds_kernel<float, false, 4, true>), grid, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        break;
      default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
    }
#undef L
  } else if (bs == 16 && vec_ok) {
    const int waves = n <= 64 ? 1 : (n <= 128 ? 2 : 4);
    dim3 grid(mb, (n + 64 * waves - 1) / (64 * waves));
    if (var >= 0 && var < 4096 && rowd && brow && crow) {
      switch (var) {
#define V(x) case x: hipLaunchKernelGGL((bsr16_f32_mfma_kernel<true, true, true, x>), grid, dim3(64 * waves), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); break;
        V(8) V(9) V(10) V(12) V(13) V(14) V(40) V(66)
#undef V
        default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
      }
    } else {
      SPMM_BSR_DISPATCH(bsr16_f32_mfma_kernel, SPMM_COMMA kBsr16Default, grid, dim3(64 * waves), ctx->stream,
                        rowd, brow, crow, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    }
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
  const int var = variant_override();
  // longest first (blocks and remainder entries) when the grid is a few
  // workgroups per slot deep (4 workgroups per CU)
  const int* ord = nullptr;
  if (const spmm_status_t st = block_row_order(ctx, mb, grid.y, brp, &ord, 4, crp, m)) {
    timing_end(ctx, slot);
    return st;
  }
  if (var == 4107)
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 3, 1, true>), grid, dim3(256), 0, ctx->stream,
                       mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else if (var == 4124)
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 3, 32, true>), grid, dim3(256), 0, ctx->stream,
                       mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else if (var == 4126)  // 32 remainder gathers in flight: 113 VGPRs, 3 workgroups per CU
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, true, 32>), grid, dim3(256), 0,
                       ctx->stream, mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else if (var == 4128)
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, true, 16>), grid, dim3(256), 0,
                       ctx->stream, mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else if (var == 4926)  // split-bf16, one k range per wave
    hipLaunchKernelGGL((bsr32_f32_lds_kernel<true, 2, 32, true, 24, true>), grid, dim3(256), 0,
                       ctx->stream, mb, n, brp, bci, bval, B, ldb, alpha, beta, C, ldc, crp, cci, cv, m, ord);
  else if (var == 4927 || (ctx->hybrid_flags & SPMM_HYBRID_SPLIT_BF16))  // wave-pair split-K
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
                               spmm_order_t orderC) {
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
  if (bs == 16 && rowd && brow && n >= 8 && n % 8 == 0 && ldb % 8 == 0 && aligned(val, 16) &&
      aligned(B, 16) && (var < 0 || var >= 4096)) {
    dim3 grid(mb, (n + 255) / 256);
    // K > 256: one workgroup per 512 columns (A read once per 512)
    const int lv = var < 0 || (var % 1000) / 100 == 2 || var / 100 == 44 || var / 100 == 45
                       ? (n >= 128 ? kBsr16F16Cs : kBsr16F16LdsDefault)
                       : var;
#define L(D)                                                                                      \
  if (crow) hipLaunchKernelGGL((bsr16_lds_kernel<_Float16, true, D>), grid, dim3(256), 0,          \
                               ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
  else hipLaunchKernelGGL((bsr16_lds_kernel<_Float16, false, D>), grid, dim3(256), 0, ctx->stream,  \
                          mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    switch (lv) {
      case 4099: L(3) break;
      case 4100: L(4) break;
      case 4102: L(6) break;
      case 4107:  // + 8: XCD-contiguous block rows
        if (crow) hipLaunchKernelGGL((bsr16_lds_kernel<_Float16, true, 3, true>), grid, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        else hipLaunchKernelGGL((bsr16_lds_kernel<_Float16, false, 3, true>), grid, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        break;
#define CM(V, ...)                                                                                  \
  case V:                                                                                           \
    if (crow) hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, true, __VA_ARGS__>), grid, dim3(256), 0, \
                                 ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
    else hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, false, __VA_ARGS__>), grid, dim3(256), 0,     \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);   \
    break;
      CM(4625, 2, 5) CM(4636, 3, 6) CM(4626, 2, 6) CM(4646, 4, 6)  // column-masked, 46 D DA
      CM(4725, 2, 5, 8) CM(4724, 2, 4, 8)  // 47 D DA: + at least 8 waves per SIMD (<= 64 registers)
      // 48 D DA: 512 output columns per workgroup (8 tiles per wave; A once per 512 columns)
#define CM512(V, ...)                                                                               \
  case V: {                                                                                         \
    const dim3 g5(mb, (n + 511) / 512);                                                             \
    if (crow) hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, true, __VA_ARGS__, 512>), g5, dim3(256), \
                                 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); \
    else hipLaunchKernelGGL((bsr16_cm_kernel<_Float16, false, __VA_ARGS__, 512>), g5, dim3(256), 0,  \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);   \
    break;                                                                                          \
  }
      CM512(4825, 2, 5, 1) CM512(4826, 2, 6, 1) CM512(4836, 3, 6, 1) CM512(4824, 2, 4, 1)
#undef CM512
      // column stream (bsr16_f16_cs_kernel): 50PN = P item stages, (NA, DA) = (8, 4) (N = 1),
      // (16, 8) (N = 2), (8, 2) (N = 0)
#define CS16(V, P, A, D, COLS, ...)                                                               \
  case V: {                                                                                       \
    const int* ord = nullptr;                                                                     \
    const dim3 gc(mb, (n + COLS - 1) / COLS);                                                     \
    if (const spmm_status_t st = block_row_order(ctx, mb, gc.y, rowptr, &ord)) {                  \
      timing_end(ctx, slot);                                                                      \
      return st;                                                                                  \
    }                                                                                             \
    if (crow) hipLaunchKernelGGL((bsr16_f16_cs_kernel<true, P, A, D, COLS, ##__VA_ARGS__>), gc, dim3(64), 0, \
                                 ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, \
                                 ldc, ord, nullptr, nullptr);                                     \
    else hipLaunchKernelGGL((bsr16_f16_cs_kernel<false, P, A, D, COLS, ##__VA_ARGS__>), gc, dim3(64), 0, \
                            ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc, \
                            ord, nullptr, nullptr);                                               \
    break;                                                                                        \
  }
      CS16(5021, 2, 8, 4, 256) CS16(5031, 3, 8, 4, 256) CS16(5041, 4, 8, 4, 256)
      CS16(5022, 2, 16, 8, 256) CS16(5032, 3, 16, 8, 256) CS16(5020, 2, 8, 2, 256)
      // 51PN: 128 output columns per wave (4-KB item stages)
      CS16(5121, 2, 8, 4, 128) CS16(5131, 3, 8, 4, 128) CS16(5141, 4, 8, 4, 128)
      CS16(5151, 5, 8, 4, 128)
      // 53xx: pending capacity 48: 5304 = P 2, NA 4, DA 0 (19.7 KB: 8 waves per CU);
      // 5308 = P 2, NA 8, DA 4; 5334 = P 3, NA 4, DA 0
      CS16(5304, 2, 4, 0, 256, 48) CS16(5308, 2, 8, 4, 256, 48) CS16(5334, 3, 4, 0, 256, 48)
      // diagnostics (wrong results): 970D = 5021 with DIAG D
      CS16(9701, 2, 8, 4, 256, 64, 1) CS16(9702, 2, 8, 4, 256, 64, 2) CS16(9704, 2, 8, 4, 256, 64, 4)
      CS16(9708, 2, 8, 4, 256, 64, 8) CS16(9706, 2, 8, 4, 256, 64, 6) CS16(9715, 2, 8, 4, 256, 64, 15)
      // 60PN: 50PN with full-line copies (FLC)
      CS16(6021, 2, 8, 4, 256, 64, 0, false, true)
      // 61PN: 50PN with two whole rows per 16-B copy (FLR)
      CS16(6121, 2, 8, 4, 256, 64, 0, false, false, true) CS16(6131, 3, 8, 4, 256, 64, 0, false, false, true)
      CS16(6122, 2, 16, 8, 256, 64, 0, false, false, true) CS16(6104, 2, 4, 0, 256, 48, 0, false, false, true)
      CS16(6120, 2, 8, 2, 256, 64, 0, false, false, true)
#undef CS16
      // 63xx: 61xx with the column tiles of a block row side by side on one XCD (TT)
#define CS16T(V, P, A, D, COLS, ...)                                                              \
  case V: {                                                                                       \
    const int* ord = nullptr;                                                                     \
    const int nt = (n + COLS - 1) / COLS;                                                         \
    if (const spmm_status_t st = block_row_order(ctx, mb, nt, rowptr, &ord)) {                    \
      timing_end(ctx, slot);                                                                      \
      return st;                                                                                  \
    }                                                                                             \
    if (crow) hipLaunchKernelGGL((bsr16_f16_cs_kernel<true, P, A, D, COLS, ##__VA_ARGS__, true>), \
                                 dim3(mb * nt), dim3(64), 0, ctx->stream, mb, n, rowptr, colind,  \
                                 val, B, ldb, alpha, beta, C, ldc, ord, nullptr, nullptr);        \
    else hipLaunchKernelGGL((bsr16_f16_cs_kernel<false, P, A, D, COLS, ##__VA_ARGS__, true>),     \
                            dim3(mb * nt), dim3(64), 0, ctx->stream, mb, n, rowptr, colind, val,  \
                            B, ldb, alpha, beta, C, ldc, ord, nullptr, nullptr);                  \
    break;                                                                                        \
  }
      CS16T(6304, 2, 4, 0, 256, 48, 0, false, false, true)
      CS16T(6321, 2, 8, 4, 256, 64, 0, false, false, true)
#undef CS16T
      // item stream (bsr16_f16_is_kernel): 55PR = P item stages, R records ahead, 256
      // columns; 56PR: 128 columns. First launch: the builder (the column stream's walk,
      // NA = 8, DA = 4) into the workspace.
#define IS16(V, P, R, COLS)                                                                       \
  case V: {                                                                                       \
    const int* ord = nullptr;                                                                     \
    const dim3 gc(mb, (n + COLS - 1) / COLS);                                                     \
    const size_t rec_bytes = (size_t)nnzb * kIsRec;                                               \
    spmm_status_t st = spmm::ensure_scratch(ctx, rec_bytes + 4 * (size_t)mb);                     \
    if (st == SPMM_STATUS_SUCCESS) st = block_row_order(ctx, mb, gc.y, rowptr, &ord);             \
    if (st != SPMM_STATUS_SUCCESS) {                                                              \
      timing_end(ctx, slot);                                                                      \
      return st;                                                                                  \
    }                                                                                             \
    char* const recs = reinterpret_cast<char*>(ctx->scratch);                                     \
    int* const nit = reinterpret_cast<int*>(recs + rec_bytes);                                    \
    hipLaunchKernelGGL((bsr16_f16_cs_kernel<true, 2, 8, 4, 256, 64, 0, true>), dim3(mb), dim3(64), \
                       0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,   \
                       nullptr, recs, nit);                                                       \
    if (crow) hipLaunchKernelGGL((bsr16_f16_is_kernel<true, P, R, COLS>), gc, dim3(64), 0,        \
                                 ctx->stream, mb, n, rowptr, recs, nit, B, ldb, alpha, beta, C,   \
                                 ldc, ord);                                                       \
    else hipLaunchKernelGGL((bsr16_f16_is_kernel<false, P, R, COLS>), gc, dim3(64), 0,            \
                            ctx->stream, mb, n, rowptr, recs, nit, B, ldb, alpha, beta, C, ldc,   \
                            ord);                                                                 \
    break;                                                                                        \
  }
      IS16(5522, 2, 2, 256) IS16(5533, 3, 3, 256) IS16(5644, 4, 4, 128)
#undef IS16
      // 57D0 / 58D0: register-staged item stream (bsr16_f16_isr_kernel), D items in flight,
      // 256 / 128 columns
#define IS16R(V, D, COLS, ...)                                                                    \
  case V: {                                                                                       \
    const int* ord = nullptr;                                                                     \
    const dim3 gc(mb, (n + COLS - 1) / COLS);                                                     \
    const size_t rec_bytes = (size_t)nnzb * kIsRec;                                               \
    spmm_status_t st = spmm::ensure_scratch(ctx, rec_bytes + 4 * (size_t)mb);                     \
    if (st == SPMM_STATUS_SUCCESS) st = block_row_order(ctx, mb, gc.y, rowptr, &ord);             \
    if (st != SPMM_STATUS_SUCCESS) {                                                              \
      timing_end(ctx, slot);                                                                      \
      return st;                                                                                  \
    }                                                                                             \
    char* const recs = reinterpret_cast<char*>(ctx->scratch);                                     \
    int* const nit = reinterpret_cast<int*>(recs + rec_bytes);                                    \
    hipLaunchKernelGGL((bsr16_f16_cs_kernel<true, 2, 8, 4, 256, 64, 0, true>), dim3(mb), dim3(64), \
                       0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc,   \
                       nullptr, recs, nit);                                                       \
    if (crow) hipLaunchKernelGGL((bsr16_f16_isr_kernel<true, D, COLS, ##__VA_ARGS__>), gc, dim3(64), 0, \
                                 ctx->stream, mb, n, rowptr, recs, nit, B, ldb, alpha, beta, C,   \
                                 ldc, ord);                                                       \
    else hipLaunchKernelGGL((bsr16_f16_isr_kernel<false, D, COLS, ##__VA_ARGS__>), gc, dim3(64), 0, \
                            ctx->stream, mb, n, rowptr, recs, nit, B, ldb, alpha, beta, C, ldc,   \
                            ord);                                                                 \
    break;                                                                                        \
  }
      IS16R(5710, 1, 256) IS16R(5720, 2, 256) IS16R(5840, 4, 128)
      // 59D0: the same with full-line B loads (one 512-B row per load instruction)
      IS16R(5910, 1, 256, true) IS16R(5920, 2, 256, true)
#undef IS16R
#undef CM
      case 4303: case 4304: {  // block-row pairs sharing B panels, D = 3 / 4
        const dim3 gp((mb + 1) / 2, (n + 255) / 256);
        if (lv == 4303) {
          if (crow) hipLaunchKernelGGL((bsr16_f16_pair_kernel<true, 3>), gp, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
          else hipLaunchKernelGGL((bsr16_f16_pair_kernel<false, 3>), gp, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        } else {
          if (crow) hipLaunchKernelGGL((bsr16_f16_pair_kernel<true, 4>), gp, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
          else hipLaunchKernelGGL((bsr16_f16_pair_kernel<false, 4>), gp, dim3(256), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
        }
        break;
      }
      default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
    }
#undef L
  } else if (bs == 16 && vec_ok) {
    const int waves = n <= 64 ? 1 : (n <= 128 ? 2 : 4);
    dim3 grid(mb, (n + 64 * waves - 1) / (64 * waves));
    if (var >= 0 && var < 4096 && rowd && brow && crow) {
      switch (var) {
#define V(x) case x: hipLaunchKernelGGL((bsr16_f16_mfma_kernel<true, true, true, x>), grid, dim3(64 * waves), 0, ctx->stream, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc); break;
        V(8) V(9) V(10) V(12) V(13) V(14) V(40) V(66)
#undef V
        default: timing_end(ctx, slot); return SPMM_STATUS_INVALID_VALUE;
      }
    } else {
      SPMM_BSR_DISPATCH(bsr16_f16_mfma_kernel, SPMM_COMMA kBsr16F16Default, grid, dim3(64 * waves), ctx->stream,
                        rowd, brow, crow, mb, n, rowptr, colind, val, B, ldb, alpha, beta, C, ldc);
    }
  } else {
    dim3 grid(mb, (n + 63) / 64);
    hipLaunchKernelGGL(bsr_generic_kernel<_Float16>, grid, dim3(256), 0, ctx->stream, mb, n, bs,
                       rowd, rowptr, colind, val, B, ldb, brow, alpha, beta, C, ldc, crow);
  }
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

}  // namespace spmm
