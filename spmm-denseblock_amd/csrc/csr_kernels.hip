// csr_kernels.hip — Path A: CSR x dense on gfx950 (MI355X).
//
// Replaces the GE-SpMM kernels of the reference (gespmm_csrmm.h:95-166,
// spmm_test2, dispatched by gespmm_csrmm -> spmmWrapper(2, 8, ...) at
// gespmm_csrmm.h:422-426) and the legacy cusparseScsrmm/csrmm2 calls.
//
// Design:
//  * Merge-path work split. The reference gives each CSR row to one warp
//    (gespmm_csrmm.h:105), so a power-law hub row (ogbn-products max degree
//    ~17k) serialises on one warp while short rows idle lanes. Here the
//    (rows + nnz) merge path is cut into equal pieces, one per wave64; each
//    wave finds its start/end coordinates with a 32-ary cooperative search
//    on rowptr (5 dependent loads for 2.4M rows), walks its nnz range and
//    emits every row that ends inside it. A row split over several waves is
//    finished in the same launch by the last of them to arrive (split_row_*
//    below: partials in wave order, deterministic, one ticket atomic per
//    wave and split row).
//  * One nnz per wave-instruction. All 64 lanes gather the same B row: lane l
//    owns columns [VEC*l, VEC*l+VEC) of a 64*VEC-wide column tile, so a
//    gather is one coalesced 256/512/1024-byte global_load_dword{,x2,x4}
//    whose row base is wave-uniform (v_readlane -> SGPR, saddr addressing).
//    colind/val are read 64 at a time with one coalesced vector load each
//    and broadcast with v_readlane; no LDS is needed because nothing
//    gathered is reused inside the wave (a LDS round trip would be pure
//    overhead, cdna_hip_programming.md App. B "GEMV" row).
//  * Latency hiding: B rows are software-pipelined in groups of U=8 nnz,
//    loads for group g+1 issued before group g is consumed, so up to 16 row
//    gathers are in flight per wave across row boundaries.
//  * Each output element is a sequential fp32 FMA chain in CSR order, like
//    the reference's `acc += val * B[...]` (gespmm_csrmm.h:124-129, contracted
//    to FMA by nvcc): rows that a single wave finishes are bit-identical to
//    the sequential oracle; rows split across waves differ only by the
//    association of the carry sum.
#include <hip/hip_runtime.h>

#include <climits>

#include "context.hpp"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerWG = 4;
constexpr int kWG = kWave * kWavesPerWG;
constexpr int kU = 8;            // nnz per pipeline group
constexpr int kR = 4;            // colind/val registers per lane per chunk
constexpr int kChunk = kWave * kR / kU;  // groups per chunk (32)
// the merge-path grid's floor on items per wave: below waves_per_cu x CUs waves a small
// matrix gets more, shorter waves (arxiv stand-in, K = 128: 0.0868 -> 0.0849 ms at 256;
// 128 ties, profiles/r04d/csr_grid.jsonl)
constexpr int kMinItemsPerWave = 256;
constexpr int kGroupMaxK = 64;  // K handled by csr_group_kernel

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VEC> struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef f32x2 T; };
template <> struct Vec<4> { typedef f32x4 T; };

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T vload(const float* p) {
  return *reinterpret_cast<const typename Vec<VEC>::T*>(p);
}
template <int VEC>
__device__ __forceinline__ void vstore(float* p, typename Vec<VEC>::T v) {
  *reinterpret_cast<typename Vec<VEC>::T*>(p) = v;
}
template <int VEC>
__device__ __forceinline__ float vget(const typename Vec<VEC>::T& v, int c) {
  if constexpr (VEC == 1) return v; else return v[c];
}
template <int VEC>
__device__ __forceinline__ void vset(typename Vec<VEC>::T& v, int c, float x) {
  if constexpr (VEC == 1) v = x; else v[c] = x;
}

// One B-row piece by a raw buffer load with cache policy AUX (0 default, 2 nt).
template <int VEC, int AUX>
__device__ __forceinline__ typename Vec<VEC>::T bload(__amdgpu_buffer_rsrc_t rs, int off,
                                                      int soff = 0) {
  if constexpr (VEC == 1) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, soff, AUX));
  } else if constexpr (VEC == 2) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, soff, AUX));
  } else {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, AUX));
  }
}

// Waits for a pending load into `x` right here. Used on the (rare) reload
// paths so that the common path that merges with them after a branch does
// not inherit a conservative vmcnt(0) for the reloaded register.
template <typename T>
__device__ __forceinline__ void settle(T& x) {
  asm volatile("" : "+v"(x));
}

__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// x from lane (l - N) mod 16 of the same 16-lane row (DPP row_ror:N).
template <int N>
__device__ __forceinline__ float dpp_ror(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x120 + N, 0xF, 0xF, false));
}
__device__ __forceinline__ float rdlanef(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Pieces: the association of a row's sum, a function of the row alone
// (DESIGN.md §3c). A row of L nonzeros is summed as consecutive pieces of
//   T(L) = max(kPieceMin, ceil(L / kMaxPieces))
// nonzeros counted from the row's first nonzero, each a sequential fp32 FMA
// chain from zero in CSR order, and the pieces are added left to right from -0:
//   x = ((-0 + p_0) + p_1) + ... + p_{np-1},   C = epi(x)
// (-0 + p = p bit for bit, so a row of at most kPieceMin nonzeros is the
// reference's own sequential chain, gespmm_csrmm.h:124-129). Merge-path wave
// boundaries are moved onto piece boundaries (snap_cut), so every piece is
// summed by one wave, and C does not depend on the grid, on the rows around
// the row (shards, chunks) or on the entry point.
constexpr int kPieceMin = 128;
// 64 pieces at most (16 in the first form: a hub row's pieces of ceil(L / 16) nonzeros put
// up to 3.1x the mean share in one wave on the arxiv stand-in, 1.4x at 64)
constexpr int kPiecesLog = 6;
constexpr int kMaxPieces = 1 << kPiecesLog;

__device__ __forceinline__ int piece_len(int L) {
  return max(kPieceMin, (int)(((unsigned)L + (kMaxPieces - 1)) >> kPiecesLog));
}

// The merge-path point (i, j) of a wave boundary (i row ends and j nonzeros
// consumed), moved off any piece: a cut strictly inside row i goes down to the
// piece boundary at or before it (the row's start for a one-piece row), and a
// cut between the row's last nonzero and its end marker moves past the marker.
// Both waves of a boundary apply it to the same diagonal, so they agree.
__device__ __forceinline__ void snap_cut(const int* __restrict__ rowptr, int rp0, int m, int& i,
                                         int& j) {
  if (i >= m) return;
  const int rs = rowptr[i] - rp0;
  if (j <= rs) return;
  const int re = rowptr[i + 1] - rp0;
  if (j >= re) {
    ++i;
    j = re;
    return;
  }
  const int T = piece_len(re - rs);
  j = rs + (j - rs) / T * T;
}

// Split rows. A row whose pieces lie in several waves is finished by the last
// of them to arrive, in the same launch:
//  * each of its waves stores every piece it summed in the row's piece slots,
//    slot (key, k): key = tile * nwaves + the wave of the row's start diagonal
//    ((row + start) / per, unique among the launch's split rows), k = the
//    piece number;
//  * after its stores have completed (s_waitcnt vmcnt(0)) each wave adds its
//    piece count to the row's ticket, tickets[key] (an agent-scope atomic), and
//    the wave whose add completes the row's np pieces resets the ticket and
//    writes C = epi(((-0 + s_0) + s_1) + ...), the arithmetic of a row that one
//    wave sums whole.
// The slots cross workgroups (and XCDs) by MI355X_MICROARCH.md's counter
// hand-off: sc1 stores and sc1 loads of every handed-off word, each storing
// wave's vmcnt(0) before its add, the last adder loading only after its add
// has returned. Tickets are zero between launches (tickets of the handle,
// never shared with other buffers).
__device__ __forceinline__ void st_sc1(float* p, float x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Adds this wave's `add` pieces to *t (lane 0); true in the wave whose add
// completes `count`, which also resets *t for the next launch.
__device__ __forceinline__ bool split_row_arrive(int* t, int add, int count, int lane) {
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(t, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readlane(old, 0);
  if (old + add != count) return false;
  if (lane == 0) __hip_atomic_store(t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
// Piece slots of the split rows: kMaxPieces slots of `stride` floats per key
// (column tile x wave): stride = the launch's column-tile width (kWave * VEC;
// kWave for the K <= 64 group kernel). The host sizes the array for the widest
// grid at that width (csrmm_carry_bytes).
struct SplitWs {
  float* slots;
  int stride;
};

// Merge-path search for two diagonals at once: lanes 0-31 search d0, lanes
// 32-63 search d1. A[i] = rowptr[i+1]-rp0 (row-end offsets), B[j] = j.
// Returns (per lane) the number of row ends consumed before the diagonal.
__device__ __forceinline__ int merge_search2(const int* __restrict__ rowptr, int rp0, int m,
                                             long long nnz, long long d0, long long d1,
                                             int lane) {
  const long long d = lane < 32 ? d0 : d1;
  int lo = (int)max(0LL, d - nnz);
  int hi = (int)min(d, (long long)m);
  const int t = lane & 31;
  while (true) {
    const int len = hi - lo;
    const bool active = len > 0;
    if (!__any(active)) break;
    const int p = lo + (int)(((long long)(t + 1) * len) / 33);
    bool pred = false;
    if (active) {
      const long long a = (long long)rowptr[p + 1] - rp0;
      pred = a <= d - p - 1;
    }
    const unsigned long long mask = __ballot(pred);
    const unsigned half = lane < 32 ? (unsigned)mask : (unsigned)(mask >> 32);
    const int c = __popc(half);
    if (active) {
      const int nlo = (c == 0) ? lo : lo + (int)(((long long)c * len) / 33) + 1;
      const int nhi = (c == 32) ? hi : lo + (int)(((long long)(c + 1) * len) / 33);
      lo = nlo;
      hi = nhi;
    }
  }
  return lo;
}

// A wave's range of the merge path after the snap, and what it shares with its
// neighbours: [(i0, j0), (i1, j1)); row i0 began in an earlier wave (head),
// row i1 continues past this wave (carry; j1 then lies strictly inside it).
struct WaveRange {
  int i0, j0, i1, j1;
  int rs0;       // start of row i0 (relative nonzero index)
  int rs1, re1;  // start / end of row i1 (when carry)
  bool head, carry;
};

__device__ __forceinline__ WaveRange wave_range(const int* __restrict__ rowptr, int rp0, int m,
                                                long long nnz, long long d0, long long d1,
                                                int lane) {
  const int ires = merge_search2(rowptr, rp0, m, nnz, d0, d1, lane);
  WaveRange r;
  r.i0 = __builtin_amdgcn_readlane(ires, 0);
  r.i1 = __builtin_amdgcn_readlane(ires, 32);
  r.j0 = (int)(d0 - r.i0);
  r.j1 = (int)(d1 - r.i1);
  snap_cut(rowptr, rp0, m, r.i0, r.j0);
  snap_cut(rowptr, rp0, m, r.i1, r.j1);
  r.rs0 = r.i0 < m ? rowptr[r.i0] - rp0 : 0;
  r.rs1 = r.i1 < m ? rowptr[r.i1] - rp0 : 0;
  r.carry = r.i1 < m && r.j1 > r.rs1;
  r.re1 = r.carry ? rowptr[r.i1 + 1] - rp0 : 0;
  r.head = r.i0 < r.i1 && r.rs0 < r.j0;
  return r;
}

// Per-row piece state of a wave (wave-uniform scalars). The wave's events
// are row ends (cur_end) and piece boundaries inside a row (next_pb), both
// relative nonzero indices; ev is the nearer one. A split row's pieces go to
// its slots (key), any other row's are added into the running sum.
struct PieceState {
  int cur_end;   // end of row i (INT_MAX for the carry row)
  int re;        // real end of row i
  int T;         // piece length of row i
  int pk;        // current piece number
  int next_pb;   // next piece boundary inside row i (INT_MAX: none)
  int ev;        // min(cur_end, next_pb)
  bool split;    // row i is split: pieces to the slots
  int stored;    // pieces of row i this wave has stored
  size_t key;    // ticket index of row i (split rows)
  __device__ __forceinline__ void begin(int rs, int re_, int cur_end_, int jfirst) {
    cur_end = cur_end_;
    re = re_;
    T = piece_len(re_ - rs);
    pk = jfirst > rs ? (jfirst - rs) / T : 0;
    const unsigned nb = (unsigned)rs + (unsigned)(pk + 1) * (unsigned)T;
    next_pb = nb < (unsigned)re_ ? (int)nb : INT_MAX;
    ev = min(cur_end, next_pb);
    stored = 0;
  }
  __device__ __forceinline__ void next_piece() {
    ++pk;
    const unsigned nb = (unsigned)next_pb + (unsigned)T;
    next_pb = nb < (unsigned)re ? (int)nb : INT_MAX;
    ev = min(cur_end, next_pb);
  }
  __device__ __forceinline__ int npieces(int rs) const { return (re - rs + T - 1) / T; }
};

template <int VEC, bool NT, int HOT = 0>
__global__ __launch_bounds__(kWG) void csr_mergepath_kernel(
    int m, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, int base, const float* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, SplitWs sws, int* __restrict__ tickets,
    int nwaves) {
  typedef typename Vec<VEC>::T vec;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
  if (w >= nwaves) return;
  const int ct = blockIdx.y;
  const int tile0 = ct * (kWave * VEC);
  const int col0 = tile0 + lane * VEC;
  const bool col_ok = col0 < n;
  const int col_ld = col_ok ? col0 : tile0;  // safe in-bounds column for masked lanes

  const int rp0 = rowptr[0];
  const long long nnz = (long long)rowptr[m] - rp0;
  const long long total = (long long)m + nnz;
  const long long per = (total + nwaves - 1) / nwaves;
  const long long d0 = min((long long)w * per, total);
  const long long d1 = min(d0 + per, total);

  const WaveRange wr = wave_range(rowptr, rp0, m, nnz, d0, d1, lane);
  const int i0 = wr.i0, i1 = wr.i1, j0 = wr.j0, j1 = wr.j1;
  if (i0 >= m) return;  // past the last row (an empty range)
  const int aoff = rp0 - base;  // array offset of relative nnz 0
  const int J = j1 - j0;
  const size_t tkeys = (size_t)ct * nwaves;  // this column tile's tickets
  const size_t sf = sws.stride;
  auto key_of = [&](int r, int rs) { return tkeys + (size_t)(((long long)r + rs) / per); };
  auto slot_p = [&](size_t key, int k) {
    return sws.slots + (key * kMaxPieces + k) * sf + lane * VEC;
  };

  // Row ends: lane l holds raw rowptr[rbase+1+l] for 64 rows, reloaded in
  // place when exhausted (one pipeline drain per 64 rows). The load is free
  // of arithmetic (clamped instead of masked, rp0 subtracted on the scalar)
  // so nothing waits for it before its first v_readlane.
  auto load_rowends = [&](int rb) -> int { return rowptr[min(rb + 1 + lane, m)]; };
  int rbase = i0;
  int rev = load_rowends(rbase);
  int i = i0;
  PieceState ps;
  if (i0 < i1) {
    const int re0 = rdlane(rev, 0) - rp0;
    ps.begin(wr.rs0, re0, re0, j0);
    ps.split = wr.head;
  } else if (wr.carry) {  // the whole range lies inside row i0 = i1
    ps.begin(wr.rs0, wr.re1, INT_MAX, j0);
    ps.split = true;
  } else {
    ps.cur_end = ps.next_pb = ps.ev = INT_MAX;
    ps.split = false;
  }
  if (ps.split) ps.key = key_of(i0, wr.rs0);

  float acc[VEC], tot[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    acc[c] = 0.f;
    tot[c] = -0.f;
  }
  // the split head row, once it has ended: its key, pieces stored here, np
  size_t head_key = 0;
  int head_stored = 0, head_np = 0;

  const float* Bb = B - (size_t)base * ldb;  // row 0 of B for 1-based colind
  float* Ct = C + col0;
  // HOT = 2 (every B offset below 4 GB): one resource for all of B, the row in soffset
  const __amdgpu_buffer_rsrc_t brs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bb), 0, 0xffffffff, 0x00020000);
  const unsigned ldb4 = 4u * (unsigned)ldb;

  auto epi_store = [&](int row, const float (&x)[VEC]) {
    float* cp = Ct + (size_t)row * ldc;
    vec out;
    if (beta == 0.f) {
#pragma unroll
      for (int c = 0; c < VEC; ++c) vset<VEC>(out, c, alpha * x[c]);
    } else {
      const vec old = vload<VEC>(col_ok ? cp : Ct);
#pragma unroll
      for (int c = 0; c < VEC; ++c)
        vset<VEC>(out, c, __builtin_fmaf(beta, vget<VEC>(old, c), alpha * x[c]));
    }
    if (col_ok) {
      if constexpr (NT) {
        // C is written once and never re-read here: stream it past the
        // caches so hub rows of B keep their L2 / MALL residency.
#pragma unroll
        for (int c = 0; c < VEC; ++c) __builtin_nontemporal_store(vget<VEC>(out, c), cp + c);
      } else {
        vstore<VEC>(cp, out);
      }
    }
  };
  auto store_piece = [&]() {
    float* sp = slot_p(ps.key, ps.pk);
#pragma unroll
    for (int c = 0; c < VEC; ++c) st_sc1(sp + c, acc[c]);
    ++ps.stored;
  };
  // the piece ending at ps.next_pb (row i continues)
  auto end_piece = [&]() {
    if (ps.split) {
      store_piece();
    } else {
#pragma unroll
      for (int c = 0; c < VEC; ++c) tot[c] = tot[c] + acc[c];
    }
#pragma unroll
    for (int c = 0; c < VEC; ++c) acc[c] = 0.f;
    ps.next_piece();
  };
  // row i ends at ps.cur_end
  auto end_row = [&]() {
    if (ps.split) {  // the split head row: its last piece to the slots
      store_piece();
      head_key = ps.key;
      head_stored = ps.stored;
      head_np = ps.pk + 1;
    } else {
      float x[VEC];
#pragma unroll
      for (int c = 0; c < VEC; ++c) x[c] = tot[c] + acc[c];
      epi_store(i, x);
    }
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      acc[c] = 0.f;
      tot[c] = -0.f;
    }
  };
  auto advance_row = [&]() {
    const int rs = ps.cur_end;  // the row just ended here
    ++i;
    if (i - rbase == kWave) {
      rbase += kWave;
      rev = load_rowends(rbase);
      settle(rev);
    }
    if (i < i1) {
      const int re = rdlane(rev, i - rbase) - rp0;
      ps.begin(rs, re, re, rs);
      ps.split = false;
    } else if (wr.carry) {
      ps.begin(rs, wr.re1, INT_MAX, rs);
      ps.split = true;
      ps.key = key_of(i, rs);
    } else {
      ps.cur_end = ps.next_pb = ps.ev = INT_MAX;
    }
  };
  auto event = [&]() {
    if (ps.cur_end <= ps.next_pb) {
      end_row();
      advance_row();
    } else {
      end_piece();
    }
  };

  // nnz are processed in groups of kU aligned to absolute array positions:
  // group g covers array indices [gs + kU*g, gs + kU*(g+1)); indices outside
  // the wave's range [A0, A1) are loaded (harmlessly) but never consumed.
  // colind/val of a chunk of kChunk groups (kChunk*kU = 256 nnz) sit in kR
  // registers per lane, lane l / register r <-> index chunk_base + kR*l + r,
  // so the register of nnz u of a group is the compile-time u % kR. They are
  // reloaded in place every kChunk groups (one pipeline drain per 256 nnz).
  const int A0 = aoff + j0, A1 = aoff + j1;
  const int gs = A0 & ~(kU - 1);
  const int G = J > 0 ? (A1 - gs + kU - 1) / kU : 0;
  if (G > 0) {
    int colv[kR];
    float valv[kR];
    auto load_chunk = [&](int c) {
      const int cb = gs + c * (kChunk * kU) + kR * lane;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int idx = min(cb + r, A1 - 1);
        if constexpr (NT) {
          colv[r] = __builtin_nontemporal_load(colind + idx);
          valv[r] = __builtin_nontemporal_load(val + idx);
        } else {
          colv[r] = colind[idx];
          valv[r] = val[idx];
        }
      }
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        settle(colv[r]);
        settle(valv[r]);
      }
    };
    float b0[kU][VEC], b1[kU][VEC];
    float v0[kU], v1[kU];  // values of the groups in flight (wave-uniform)

    auto issue = [&](float (&dst)[kU][VEC], float (&vdst)[kU], int g) {
      if ((g & (kChunk - 1)) == 0) load_chunk(g / kChunk);
      const int lb = (g & (kChunk - 1)) * (kU / kR);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int l = lb + u / kR;
        vdst[u] = rdlanef(valv[u % kR], l);
        // Wave-uniform row base (SGPRs) + per-lane column offset.
        const int cr = rdlane(colv[u % kR], l);
        const float* rowp = Bb + (size_t)(HOT ? (cr & 0x7fffffff) : cr) * ldb;
        vec x;
        if constexpr (HOT == 2) {
          // the same with the row offset in soffset (no per-row resource: 6 fewer
          // scalar instructions per nonzero)
          const int so = (int)((unsigned)(cr & 0x7fffffff) * ldb4);
          if (cr < 0)
            x = bload<VEC, 0>(brs, 4 * col_ld, so);
          else
            x = bload<VEC, 2>(brs, 4 * col_ld, so);
        } else if constexpr (HOT == 1) {
          // tagged colind (spmm_csr_hot_analysis): bit 31 marks a column whose B
          // row is worth keeping in L2 / MALL; every other row is streamed (nt), so
          // the long tail of rarely used rows does not evict the hubs (products
          // stand-in, K = 128: 4.29 -> 4.14 ms at the default 128-MB budget; sc0 /
          // sc1 cold loads change nothing, nt on every row 6.5 ms: DESIGN.md §3b).
          // Buffer loads: the cache policy is an immediate of the intrinsic, so the
          // two arms stay two instructions (plain loads were merged, nt dropped).
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(rowp), 0, 0x7fffffff, 0x00020000);
          if (cr < 0)
            x = bload<VEC, 0>(rs, 4 * col_ld);
          else
            x = bload<VEC, 2>(rs, 4 * col_ld);
        } else {
          x = vload<VEC>(rowp + col_ld);
        }
#pragma unroll
        for (int c = 0; c < VEC; ++c) dst[u][c] = vget<VEC>(x, c);
      }
    };
    auto consume = [&](float (&src)[kU][VEC], const float (&vsrc)[kU], int g) {
      const int ag = gs + g * kU;
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int a = ag + u;
        if (a >= A0 && a < A1) {
          const int j = a - aoff;
          while (ps.ev <= j) event();  // ev is INT_MAX past the last event
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[c] = __builtin_fmaf(vsrc[u], src[u][c], acc[c]);
        }
      }
    };

    issue(b0, v0, 0);
    for (int g = 0; g < G; g += 2) {
      if (g + 1 < G) issue(b1, v1, g + 1);
      consume(b0, v0, g);
      if (g + 1 < G) {
        if (g + 2 < G) issue(b0, v0, g + 2);
        consume(b1, v1, g + 1);
      }
    }
  }
  // Rows whose end marker lies at or before j1 but after the last nnz.
  while (i < i1) {
    end_row();
    advance_row();
  }
  // The carry row's pieces summed here: the last one ends at j1, a piece boundary.
  if (wr.carry && J > 0) store_piece();
  const bool carry_here = wr.carry && ps.stored > 0;
  if (!head_np && !carry_here) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces are stored
  // the last arrival of a split row writes it
  auto finish = [&](int r, size_t key, int np) {
    const float* sp = slot_p(key, 0);
    float x[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) x[c] = -0.f;
    for (int k = 0; k < np; ++k) {
#pragma unroll
      for (int c = 0; c < VEC; ++c) x[c] = x[c] + ld_sc1(sp + c);
      sp += sf;
    }
    epi_store(r, x);
  };
  if (head_np && split_row_arrive(tickets + head_key, head_stored, head_np, lane))
    finish(i0, head_key, head_np);
  if (carry_here) {
    const int np = ps.npieces(wr.rs1);
    if (split_row_arrive(tickets + ps.key, ps.stored, np, lane)) finish(i1, ps.key, np);
  }
}

// Small-K form (K <= 64, K % 4 == 0): the wave is cut into G = 64 / LPG lane
// groups of LPG lanes (LPG = 2 / 4 / 8 / 16 for K <= 8 / 16 / 32 / 64; lane l: group
// l / LPG, columns 4 (l % LPG) .. +3), each group a different nnz of the
// wave's merge-path range per step. A step is one G-row gather with per-lane
// colind / val loads instead of per-nnz v_readlane and scalar address
// arithmetic, which is what bounds the main kernel at small K.
// Each group accumulates its own partial of the current piece; at a piece or
// row end the groups before the end position are folded in and the G partials
// summed across groups (log2 G cross-lane steps). Products of a piece are thus
// summed in G interleaved chains by array position mod G — within the fp32
// bar, not bit-identical to the sequential order (SPMM_CSR_SEQUENTIAL_ROWS
// keeps the main kernel) — and the pieces are combined as in the main kernel,
// so C depends on the row and its array position mod 64 only.
template <bool NT, int LPG, int PD, bool HOT = false>
__global__ __launch_bounds__(kWG) void csr_group_kernel(
    int m, int n, const int* __restrict__ rowptr, const int* __restrict__ colind,
    const float* __restrict__ val, int base, const float* __restrict__ B, int ldb, float alpha,
    float beta, float* __restrict__ C, int ldc, SplitWs sws, int* __restrict__ tickets,
    int nwaves) {
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
  if (w >= nwaves) return;
  constexpr int G = kWave / LPG;  // nnz per step (lane groups)
  const int grp = lane / LPG;
  const int col = 4 * (lane % LPG);
  const bool col_ok = col < n;
  const int col_ld = col_ok ? col : 0;

  const int rp0 = rowptr[0];
  const long long nnz = (long long)rowptr[m] - rp0;
  const long long total = (long long)m + nnz;
  const long long per = (total + nwaves - 1) / nwaves;
  const long long d0 = min((long long)w * per, total);
  const long long d1 = min(d0 + per, total);
  const WaveRange wr = wave_range(rowptr, rp0, m, nnz, d0, d1, lane);
  const int i0 = wr.i0, i1 = wr.i1, j0 = wr.j0, j1 = wr.j1;
  if (i0 >= m) return;
  const int aoff = rp0 - base;
  const size_t sf = sws.stride;  // kWave: column c of a slot is float c
  auto key_of = [&](int r, int rs) { return (size_t)(((long long)r + rs) / per); };

  auto load_rowends = [&](int rb) -> int { return rowptr[min(rb + 1 + lane, m)]; };
  int rbase = i0;
  int rev = load_rowends(rbase);
  int i = i0;
  PieceState ps;
  if (i0 < i1) {
    const int re0 = rdlane(rev, 0) - rp0;
    ps.begin(wr.rs0, re0, re0, j0);
    ps.split = wr.head;
  } else if (wr.carry) {
    ps.begin(wr.rs0, wr.re1, INT_MAX, j0);
    ps.split = true;
  } else {
    ps.cur_end = ps.next_pb = ps.ev = INT_MAX;
    ps.split = false;
  }
  if (ps.split) ps.key = key_of(i0, wr.rs0);
  size_t head_key = 0;
  int head_stored = 0, head_np = 0;

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 tot = {-0.f, -0.f, -0.f, -0.f};
  const float* Bb = B - (size_t)base * ldb;
  // Sum of the G group partials, in every lane of the same column slot:
  // rotations inside 16-lane rows (v_add_f32_dpp row_ror: one instruction per
  // step), then the rows with two cross-lane shuffles.
  auto fold = [&](f32x4 v) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float x = v[c];
      if constexpr (LPG <= 2) x += dpp_ror<2>(x);
      if constexpr (LPG <= 4) x += dpp_ror<4>(x);
      if constexpr (LPG <= 8) x += dpp_ror<8>(x);
      x += __shfl_xor(x, 16);
      v[c] = x + __shfl_xor(x, 32);
    }
    return v;
  };
  auto store_piece = [&](const f32x4& t) {
    if (grp == 0) {
      float* sp = sws.slots + (ps.key * kMaxPieces + ps.pk) * sf + col;
#pragma unroll
      for (int c = 0; c < 4; ++c) st_sc1(sp + c, t[c]);
    }
    ++ps.stored;
  };
  auto epi_store = [&](int row, const f32x4& x) {
    if (grp == 0 && col_ok) {
      float* cp = C + (size_t)row * ldc + col;
      f32x4 out;
      if (beta == 0.f) {
#pragma unroll
        for (int c = 0; c < 4; ++c) out[c] = alpha * x[c];
      } else {
        const f32x4 old = *reinterpret_cast<const f32x4*>(cp);
#pragma unroll
        for (int c = 0; c < 4; ++c) out[c] = __builtin_fmaf(beta, old[c], alpha * x[c]);
      }
      if constexpr (NT) {
#pragma unroll
        for (int c = 0; c < 4; ++c) __builtin_nontemporal_store(out[c], cp + c);
      } else {
        *reinterpret_cast<f32x4*>(cp) = out;
      }
    }
  };
  auto end_piece = [&]() {
    const f32x4 t = fold(acc);
    if (ps.split) {
      store_piece(t);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) tot[c] = tot[c] + t[c];
    }
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    ps.next_piece();
  };
  auto end_row = [&]() {
    const f32x4 t = fold(acc);
    if (ps.split) {  // the split head row: its last piece to the slots
      store_piece(t);
      head_key = ps.key;
      head_stored = ps.stored;
      head_np = ps.pk + 1;
    } else {
      f32x4 x;
#pragma unroll
      for (int c = 0; c < 4; ++c) x[c] = tot[c] + t[c];
      epi_store(i, x);
    }
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    tot = f32x4{-0.f, -0.f, -0.f, -0.f};
  };
  auto advance_row = [&]() {
    const int rs = ps.cur_end;
    ++i;
    if (i - rbase == kWave) {
      rbase += kWave;
      rev = load_rowends(rbase);
      settle(rev);
    }
    if (i < i1) {
      const int re = rdlane(rev, i - rbase) - rp0;
      ps.begin(rs, re, re, rs);
      ps.split = false;
    } else if (wr.carry) {
      ps.begin(rs, wr.re1, INT_MAX, rs);
      ps.split = true;
      ps.key = key_of(i, rs);
    } else {
      ps.cur_end = ps.next_pb = ps.ev = INT_MAX;
      ps.split = false;
    }
  };

  // Steps of G nnz aligned to absolute array positions (as the main kernel):
  // step s covers [gs + G s, gs + G s + G); lane group g takes position + g.
  const int A0 = aoff + j0, A1 = aoff + j1;
  const int gs = A0 & ~(G - 1);
  const int S = j1 > j0 ? (A1 - gs + G - 1) / G : 0;
  auto load_idx = [&](int s, int& c, float& v) {
    const int p = min(max(gs + G * s + grp, A0), A1 - 1);  // clamped: always a valid index
    if constexpr (NT) {
      c = __builtin_nontemporal_load(colind + p);
      v = __builtin_nontemporal_load(val + p);
    } else {
      c = colind[p];
      v = val[p];
    }
  };
  auto load_b = [&](int c) {
    // hot-tagged indices (spmm_csrmm_hot_f32): the tag is dropped here; each lane
    // group gathers its own row, so a per-row policy would split every load in two
    if constexpr (HOT) c &= 0x7fffffff;
    return *reinterpret_cast<const f32x4*>(Bb + (size_t)c * ldb + col_ld);
  };
  // One step's products: groups before an event (piece or row end) inside the
  // step belong to the piece that ends there.
  auto consume = [&](int s, const f32x4& b, float v) {
    const int q0 = gs + G * s;
    const int p = q0 + grp;
    const bool ok = p >= A0 && p < A1;
    f32x4 prod;
#pragma unroll
    for (int c = 0; c < 4; ++c) prod[c] = ok ? v * b[c] : 0.f;
    // events inside the range only (ev is INT_MAX past the last one): the carry row's
    // piece boundary at j1 ends this wave's share, stored after the loop, and the
    // rows ending at j1 are emitted there too
    while (ps.ev < j1 && ps.ev - (q0 - aoff) < G) {
      const int e = ps.ev - (q0 - aoff);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool mine = grp < e;
        acc[c] += mine ? prod[c] : 0.f;
        prod[c] = mine ? 0.f : prod[c];
      }
      if (ps.cur_end <= ps.next_pb) {
        end_row();
        advance_row();
      } else {
        end_piece();
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += prod[c];
  };
  if (S > 0) {
    // Pipeline: PD B-row gathers in flight (ring slot u = s % PD holds step
    // s's row and value), indices PD steps ahead of their gather. Step
    // indices past the end are clamped (valid, never consumed).
    f32x4 bq[PD];
    float vq[PD], vi[PD];
    int ci[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      int c;
      load_idx(min(u, S - 1), c, vq[u]);
      bq[u] = load_b(c);
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) load_idx(min(PD + u, S - 1), ci[u], vi[u]);
    for (int s0 = 0; s0 < S; s0 += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        const int s = s0 + u;
        if (s >= S) break;
        const f32x4 b = bq[u];
        const float v = vq[u];
        bq[u] = load_b(ci[u]);  // step s + PD
        vq[u] = vi[u];
        load_idx(min(s + 2 * PD, S - 1), ci[u], vi[u]);
        consume(s, b, v);
      }
    }
  }
  while (i < i1) {
    end_row();
    advance_row();
  }
  if (wr.carry && j1 > j0) store_piece(fold(acc));
  const bool carry_here = wr.carry && ps.stored > 0;
  if (!head_np && !carry_here) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces are stored
  // the last arrival writes the row: lane l column l (n <= 64)
  auto finish = [&](int r, size_t key, int np) {
    const float* sp = sws.slots + key * kMaxPieces * sf + lane;
    float x = -0.f;
    for (int k = 0; k < np; ++k) {
      x = x + ld_sc1(sp);
      sp += sf;
    }
    if (lane >= n) return;
    float* cp = C + (size_t)r * ldc + lane;
    const float out = beta == 0.f ? alpha * x : __builtin_fmaf(beta, *cp, alpha * x);
    if constexpr (NT) __builtin_nontemporal_store(out, cp); else *cp = out;
  };
  if (head_np && split_row_arrive(tickets + head_key, head_stored, head_np, lane))
    finish(i0, head_key, head_np);
  if (carry_here) {
    const int np = ps.npieces(wr.rs1);
    if (split_row_arrive(tickets + ps.key, ps.stored, np, lane)) finish(i1, ps.key, np);
  }
}

// dst (cols x rows, ld_dst) = transpose(src (rows x cols, ld_src)) [+ beta*dst]
__global__ __launch_bounds__(256) void transpose_kernel(int rows, int cols,
                                                        const float* __restrict__ src,
                                                        int ld_src, float* __restrict__ dst,
                                                        int ld_dst, float beta) {
  __shared__ float tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + k][tx] = src[(size_t)r * ld_src + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < rows && c < cols) {
      float* p = dst + (size_t)c * ld_dst + r;
      const float x = tile[tx][ty + k];
      *p = (beta == 0.f) ? x : __builtin_fmaf(beta, *p, x);
    }
  }
}

// The same with 16-byte accesses on both sides (64 x 64 tiles), for any shape:
// loads go along src rows and stores along dst rows as 4-float vectors that
// need only 4-byte alignment (odd leading dimensions such as the 2,449,029
// rows of products), scalar at the matrix edges; the tile is read back down
// its columns (stride 65: conflict-free).
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
__global__ __launch_bounds__(256) void transpose4_kernel(int rows, int cols,
                                                         const float* __restrict__ src,
                                                         int ld_src, float* __restrict__ dst,
                                                         int ld_dst, float beta) {
  __shared__ float tile[64][65];
  const int t = threadIdx.x;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int q = t & 15, rb = t >> 4;  // 4-float group in a 64-wide row, first row
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rb + 16 * i, c = 4 * q;
    if (r0 + r >= rows) continue;
    const float* p = src + (size_t)(r0 + r) * ld_src + c0 + c;
    if (c0 + c + 3 < cols) {
      const f32x4u x = *reinterpret_cast<const f32x4u*>(p);
      tile[r][c] = x[0]; tile[r][c + 1] = x[1]; tile[r][c + 2] = x[2]; tile[r][c + 3] = x[3];
    } else {
      for (int e = 0; e < 4 && c0 + c + e < cols; ++e) tile[r][c + e] = p[e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = rb + 16 * i, r = 4 * q;  // dst row c0 + c, dst columns r0 + r .. + 3
    if (c0 + c >= cols || r0 + r >= rows) continue;
    float* p = dst + (size_t)(c0 + c) * ld_dst + r0 + r;
    if (r0 + r + 3 < rows) {
      f32x4u x = {tile[r][c], tile[r + 1][c], tile[r + 2][c], tile[r + 3][c]};
      if (beta != 0.f) {
        const f32x4u o = *reinterpret_cast<const f32x4u*>(p);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = __builtin_fmaf(beta, o[e], x[e]);
      }
      *reinterpret_cast<f32x4u*>(p) = x;
    } else {
      for (int e = 0; e < 4 && r0 + r + e < rows; ++e) {
        const float x = tile[r + e][c];
        p[e] = (beta == 0.f) ? x : __builtin_fmaf(beta, p[e], x);
      }
    }
  }
}

// 16-bit dst (cols x rows, ld_dst) = transpose(src (rows x cols, ld_src)):
// the fp16 B operand of the column-major BSR forms, staged row-major.
__global__ __launch_bounds__(256) void transpose16_kernel(int rows, int cols,
                                                          const uint16_t* __restrict__ src,
                                                          int ld_src, uint16_t* __restrict__ dst,
                                                          int ld_dst) {
  __shared__ uint16_t tile[32][34];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + k][tx] = src[(size_t)r * ld_src + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < rows && c < cols) dst[(size_t)c * ld_dst + r] = tile[tx][ty + k];
  }
}

// 16-bit, 64 x 64 tiles, 4 elements (8 B, 2-byte aligned) per access on both sides.
typedef uint16_t u16x4u __attribute__((ext_vector_type(4), aligned(2)));
__global__ __launch_bounds__(256) void transpose16x4_kernel(int rows, int cols,
                                                            const uint16_t* __restrict__ src,
                                                            int ld_src, uint16_t* __restrict__ dst,
                                                            int ld_dst) {
  __shared__ uint16_t tile[64][66];
  const int t = threadIdx.x;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int q = t & 15, rb = t >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rb + 16 * i, c = 4 * q;
    if (r0 + r >= rows) continue;
    const uint16_t* p = src + (size_t)(r0 + r) * ld_src + c0 + c;
    if (c0 + c + 3 < cols) {
      const u16x4u x = *reinterpret_cast<const u16x4u*>(p);
      tile[r][c] = x[0]; tile[r][c + 1] = x[1]; tile[r][c + 2] = x[2]; tile[r][c + 3] = x[3];
    } else {
      for (int e = 0; e < 4 && c0 + c + e < cols; ++e) tile[r][c + e] = p[e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = rb + 16 * i, r = 4 * q;
    if (c0 + c >= cols || r0 + r >= rows) continue;
    uint16_t* p = dst + (size_t)(c0 + c) * ld_dst + r0 + r;
    if (r0 + r + 3 < rows) {
      const u16x4u x = {tile[r][c], tile[r + 1][c], tile[r + 2][c], tile[r + 3][c]};
      *reinterpret_cast<u16x4u*>(p) = x;
    } else {
      for (int e = 0; e < 4 && r0 + r + e < rows; ++e) p[e] = tile[r + e][c];
    }
  }
}

int pick_vec(int n, const float* B, int ldb, const float* C, int ldc) {
  auto aligned = [](const void* p, int bytes) {
    return (reinterpret_cast<uintptr_t>(p) % bytes) == 0;
  };
  if (n > 128 && n % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && aligned(B, 16) && aligned(C, 16))
    return 4;
  if (n > 64 && n % 2 == 0 && ldb % 2 == 0 && ldc % 2 == 0 && aligned(B, 8) && aligned(C, 8))
    return 2;
  return 1;
}

extern "C" int spmm_csr_default_waves_per_cu(int m, int hot) {
  return !hot && m >= (1 << 20) ? 12 : 16;
}

// Waves in the merge-path grid: enough that each gets >= kMinItemsPerWave
// items, capped at the resident target (waves_per_cu x CUs) so the whole
// grid runs in one round. nnz < 0 (unknown on the host) sizes from m. The default
// target is 16 waves per CU (4 workgroups), 12 (3) from 2^20 rows on the plain kernel:
// products stand-in K = 128 4.23-4.25 ms at 12 against 4.34-4.36 at 16 (interleaved on
// one box), K = 256 even; the hot-column kernel the other way (4.30-4.31 at 12 against
// 4.17-4.18), the arxiv stand-in too (0.103 at 12 against 0.093); 10 and 14 (workgroup
// counts the CUs do not divide evenly) 4.49 / 4.63-4.68 (profiles/r06/wpc/). The
// association of every row's sum does not depend on the grid (pieces).
int csr_nwaves(spmm_context* ctx, int m, long long nnz, bool hot) {
  const int wpc = ctx->csr_waves_per_cu > 0 ? ctx->csr_waves_per_cu
                                             : spmm_csr_default_waves_per_cu(m, hot ? 1 : 0);
  const long long cap = (long long)ctx->num_cus * wpc;
  const long long total = nnz >= 0 ? (long long)m + nnz : (long long)m * 32;
#ifdef SPMM_TUNING
  static const int min_items = [] {
    const char* e = getenv("SPMM_CSR_MIN_ITEMS");  // TUNING builds only
    return e && atoi(e) > 0 ? atoi(e) : kMinItemsPerWave;
  }();
#else
  constexpr int min_items = kMinItemsPerWave;
#endif
  long long nw = (total + min_items - 1) / min_items;
  if (nw < 1) nw = 1;
  if (nw > cap) nw = cap;
  return (int)nw;
}

// ---------------------------------------------------------------------------
// spmm_csr_hot_analysis (once per matrix): which columns' B rows the gathers
// keep in the caches. Count the nonzeros of every column, histogram the counts
// (kHotBins bins, the last one open-ended), pick the count threshold that keeps
// at most hot_rows columns above it, and write colind | bit 31 for the hot ones.
// ---------------------------------------------------------------------------
constexpr int kHotBins = 8192;

__global__ __launch_bounds__(256) void col_count_kernel(long long nnz, const int* __restrict__ colind,
                                                       int base, int k, unsigned* __restrict__ cnt) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nnz;
       i += (long long)gridDim.x * 256) {
    const int c = colind[i] - base;
    if ((unsigned)c < (unsigned)k) atomicAdd(cnt + c, 1u);
  }
}

// per-workgroup LDS histogram of the counts (most columns share a few small
// counts: global atomics on those bins would serialise), flushed once
__global__ __launch_bounds__(256) void count_hist_kernel(int k, const unsigned* __restrict__ cnt,
                                                        unsigned* __restrict__ hist) {
  __shared__ unsigned h[kHotBins];
  for (int b = threadIdx.x; b < kHotBins; b += 256) h[b] = 0;
  __syncthreads();
  for (int c = blockIdx.x * 256 + threadIdx.x; c < k; c += gridDim.x * 256)
    atomicAdd(h + min(cnt[c], (unsigned)(kHotBins - 1)), 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < kHotBins; b += 256)
    if (h[b]) atomicAdd(hist + b, h[b]);
}

// thr = the smallest bin t with (columns in bins >= t) <= hot_rows; a column is
// hot iff min(count, kHotBins - 1) >= thr (thr = kHotBins: none; nonzero-free
// columns are never gathered, so thr = 0 only when every column fits)
__global__ __launch_bounds__(1024) void hot_select_kernel(const unsigned* __restrict__ hist,
                                                         long long hot_rows,
                                                         unsigned* __restrict__ thr) {
  constexpr int kPer = kHotBins / 1024;
  __shared__ unsigned long long part[1024];
  const int t = threadIdx.x;
  const int top = kHotBins - kPer * t - 1;  // thread t owns bins top .. top - kPer + 1
  unsigned long long s = 0;
  for (int j = 0; j < kPer; ++j) s += hist[top - j];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const unsigned long long v = t >= o ? part[t - o] : 0ull;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const unsigned long long above = t ? part[t - 1] : 0ull;  // columns in the bins above mine
  if (above <= (unsigned long long)hot_rows && part[t] > (unsigned long long)hot_rows) {
    unsigned long long c = above;
    int b = top;
    for (; b > top - kPer; --b) {
      if (c + hist[b] > (unsigned long long)hot_rows) break;
      c += hist[b];
    }
    *thr = (unsigned)(b + 1);
  }
  if (t == 1023 && part[t] <= (unsigned long long)hot_rows) *thr = 0u;
}

__global__ __launch_bounds__(256) void hot_tag_kernel(long long nnz, const int* __restrict__ colind,
                                                     int base, int k,
                                                     const unsigned* __restrict__ cnt,
                                                     const unsigned* __restrict__ thr,
                                                     int* __restrict__ out) {
  const unsigned t = *thr;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nnz;
       i += (long long)gridDim.x * 256) {
    const int ci = colind[i];
    const int c = ci - base;
    const bool hot = (unsigned)c < (unsigned)k && min(cnt[c], (unsigned)(kHotBins - 1)) >= t;
    out[i] = hot ? (int)((unsigned)ci | 0x80000000u) : ci;
  }
}

}  // namespace

namespace spmm {

spmm_status_t launch_csr_hot_analysis(spmm_context* ctx, int k, long long nnz, const int* colind,
                                      int base, long long hot_rows, int* colind_out) {
  // scratch: counts (k words), histogram, threshold
  const size_t cnt_bytes = ((size_t)k * 4 + 255) & ~(size_t)255;
  spmm_status_t st = ensure_scratch(ctx, cnt_bytes + kHotBins * 4 + 256);
  if (st != SPMM_STATUS_SUCCESS) return st;
  unsigned* cnt = static_cast<unsigned*>(ctx->scratch);
  unsigned* hist = reinterpret_cast<unsigned*>(static_cast<char*>(ctx->scratch) + cnt_bytes);
  unsigned* thr = hist + kHotBins;
  hipError_t e = hipMemsetAsync(cnt, 0, cnt_bytes + kHotBins * 4, ctx->stream);
  if (e != hipSuccess) return from_hip(e);
  const int grid = ctx->num_cus * 8;
  hipLaunchKernelGGL(col_count_kernel, dim3(grid), dim3(256), 0, ctx->stream, nnz, colind, base, k,
                     cnt);
  hipLaunchKernelGGL(count_hist_kernel, dim3(ctx->num_cus), dim3(256), 0, ctx->stream, k, cnt,
                     hist);
  hipLaunchKernelGGL(hot_select_kernel, dim3(1), dim3(1024), 0, ctx->stream, hist, hot_rows, thr);
  hipLaunchKernelGGL(hot_tag_kernel, dim3(grid), dim3(256), 0, ctx->stream, nnz, colind, base, k,
                     cnt, thr, colind_out);
  return from_hip(hipGetLastError());
}

namespace {
// Floats of the piece slots: kMaxPieces slots of one column tile's width per
// (column tile, wave) at the capped wave count. The tiles of a launch cover
// roundup(n, 64 * VEC) columns, at most the width below for any VEC
// pick_vec can choose at this n (VEC 4 only past 128 columns, VEC 2 past 64),
// and the group kernel's single tile of kWave floats is within it too, so one
// size serves every launch of this n.
size_t split_array_floats(spmm_context* ctx, int n) {
  const int wpc = ctx->csr_waves_per_cu > 0 ? ctx->csr_waves_per_cu : 16;
  const size_t nw = (size_t)ctx->num_cus * wpc;  // the grid's cap (csr_nwaves)
  const size_t un = (size_t)n;
  const size_t width = n > 128 ? (un + 255) & ~(size_t)255 : (n > 64 ? 128 : 64);
  return nw * kMaxPieces * width;
}
}  // namespace

size_t csrmm_carry_bytes(spmm_context* ctx, int m, int n) {
  (void)m;  // the grid does not depend on m or nnz beyond the cap: size it for the cap
  return split_array_floats(ctx, n) * sizeof(float) + 256;
}

spmm_status_t launch_csrmm_rowmajor(spmm_context* ctx, int m, int n, const int* rowptr,
                                    const int* colind, const float* val, int base,
                                    const float* B, int ldb, float alpha, float beta, float* C,
                                    int ldc, void* carry_ws, int nnz_hint, int hot) {
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  const int vec = pick_vec(n, B, ldb, C, ldc);
  const int tile = kWave * vec;
  const int ntiles = (n + tile - 1) / tile;
  const int nw = csr_nwaves(ctx, m, nnz_hint, hot != 0);
  dim3 grid((nw + kWavesPerWG - 1) / kWavesPerWG, ntiles);
  dim3 block(kWG);
  // split rows: piece slots in the workspace (sized by csrmm_carry_bytes for the
  // largest grid), tickets of the handle (zero between launches)
  SplitWs sws;
  sws.slots = static_cast<float*>(carry_ws);
  sws.stride = tile;
  if (spmm_status_t st = ensure_tickets(ctx, (size_t)nw * ntiles)) return st;
  int* tickets = ctx->tickets;
  const int slot = timing_begin(ctx);
  const bool nt = (ctx->csr_flags & SPMM_CSR_NT_STREAMS) != 0;
  const bool grouped = n <= kGroupMaxK && n % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 &&
                      reinterpret_cast<uintptr_t>(B) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(C) % 16 == 0 &&
                      (ctx->csr_flags & SPMM_CSR_SEQUENTIAL_ROWS) == 0;
  if (grouped) {
    sws.stride = kWave;  // one column tile: lane l owns column l (n <= 64)
    dim3 g8((nw + kWavesPerWG - 1) / kWavesPerWG, 1);
#ifdef SPMM_TUNING
    static const int pd_env = [] {
      const char* e = getenv("SPMM_CSR_GROUP_PD");  // TUNING builds only
      return e ? atoi(e) : 0;
    }();
#else
    constexpr int pd_env = 0;
#endif
#define SPMM_LAUNCH_GRP_PD(L, PD)                                                              \
  if (hot)                                                                                     \
    hipLaunchKernelGGL((csr_group_kernel<true, L, PD, true>), g8, block, 0, ctx->stream, m, n,  \
                       rowptr, colind, val, base, B, ldb, alpha, beta, C, ldc, sws, tickets,    \
                       nw);                                                                     \
  else if (nt)                                                                                 \
    hipLaunchKernelGGL((csr_group_kernel<true, L, PD>), g8, block, 0, ctx->stream, m, n,        \
                       rowptr, colind, val, base, B, ldb, alpha, beta, C, ldc, sws, tickets,    \
                       nw);                                                                     \
  else                                                                                         \
    hipLaunchKernelGGL((csr_group_kernel<false, L, PD>), g8, block, 0, ctx->stream, m, n,       \
                       rowptr, colind, val, base, B, ldb, alpha, beta, C, ldc, sws, tickets,    \
                       nw);
    // gathers in flight per wave: 1 at K <= 16, where a gather costs a whole
    // 128-B line and depth is no help; 2 at K = 32 (1.21 vs 1.35 ms on
    // products); 4 at K = 48 / 64 (2.19 / 2.27 ms vs 2.33 / 2.37 for the
    // main kernel)
    const int pd = pd_env > 0 ? pd_env : (n <= 16 ? 1 : (n <= 32 ? 2 : 4));
#define SPMM_LAUNCH_GRP(L)                                                                     \
  if (pd == 1) { SPMM_LAUNCH_GRP_PD(L, 1) }                                                    \
  else if (pd == 4) { SPMM_LAUNCH_GRP_PD(L, 4) }                                               \
  else { SPMM_LAUNCH_GRP_PD(L, 2) }
    // lanes per nnz: 4 columns each, so 2 / 4 / 8 / 16 lanes cover K <= 8 / 16 / 32 / 64
    if (n <= 8) {
      SPMM_LAUNCH_GRP(2)
    } else if (n <= 16) {
      SPMM_LAUNCH_GRP(4)
    } else if (n <= 32) {
      SPMM_LAUNCH_GRP(8)
    } else {
      SPMM_LAUNCH_GRP(16)
    }
#undef SPMM_LAUNCH_GRP
#undef SPMM_LAUNCH_GRP_PD
    timing_end(ctx, slot);
    return from_hip(hipGetLastError());
  }
#define SPMM_LAUNCH_MP(V, N)                                                                   \
  hipLaunchKernelGGL((csr_mergepath_kernel<V, N>), grid, block, 0, ctx->stream, m, n, rowptr, \
                     colind, val, base, B, ldb, alpha, beta, C, ldc, sws, tickets, nw)
#define SPMM_LAUNCH_HOT(V, H)                                                                  \
  hipLaunchKernelGGL((csr_mergepath_kernel<V, true, H>), grid, block, 0, ctx->stream, m, n,    \
                     rowptr, colind, val, base, B, ldb, alpha, beta, C, ldc, sws, tickets, nw)
  if (hot == 2) {
    if (vec == 4) SPMM_LAUNCH_HOT(4, 2); else if (vec == 2) SPMM_LAUNCH_HOT(2, 2); else SPMM_LAUNCH_HOT(1, 2);
  } else if (hot) {
    if (vec == 4) SPMM_LAUNCH_HOT(4, 1); else if (vec == 2) SPMM_LAUNCH_HOT(2, 1); else SPMM_LAUNCH_HOT(1, 1);
  } else if (vec == 4) {
    if (nt) SPMM_LAUNCH_MP(4, true); else SPMM_LAUNCH_MP(4, false);
  } else if (vec == 2) {
    if (nt) SPMM_LAUNCH_MP(2, true); else SPMM_LAUNCH_MP(2, false);
  } else {
    if (nt) SPMM_LAUNCH_MP(1, true); else SPMM_LAUNCH_MP(1, false);
  }
#undef SPMM_LAUNCH_MP
#undef SPMM_LAUNCH_HOT
  timing_end(ctx, slot);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_transpose(spmm_context* ctx, int rows, int cols, const float* src,
                               int ld_src, float* dst, int ld_dst, float beta) {
  if (rows == 0 || cols == 0) return SPMM_STATUS_SUCCESS;
  if ((rows + 63) / 64 <= 65535) {
    dim3 grid((cols + 63) / 64, (rows + 63) / 64);
    hipLaunchKernelGGL(transpose4_kernel, grid, dim3(256), 0, ctx->stream, rows, cols, src,
                       ld_src, dst, ld_dst, beta);
    return from_hip(hipGetLastError());
  }
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, ctx->stream, rows, cols, src, ld_src,
                     dst, ld_dst, beta);
  return from_hip(hipGetLastError());
}

spmm_status_t launch_transpose16(spmm_context* ctx, int rows, int cols, const uint16_t* src,
                                 int ld_src, uint16_t* dst, int ld_dst) {
  if (rows == 0 || cols == 0) return SPMM_STATUS_SUCCESS;
  if ((rows + 63) / 64 <= 65535 && reinterpret_cast<uintptr_t>(src) % 2 == 0) {
    dim3 grid((cols + 63) / 64, (rows + 63) / 64);
    hipLaunchKernelGGL(transpose16x4_kernel, grid, dim3(256), 0, ctx->stream, rows, cols, src,
                       ld_src, dst, ld_dst);
    return from_hip(hipGetLastError());
  }
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, ctx->stream, rows, cols, src, ld_src,
                     dst, ld_dst);
  return from_hip(hipGetLastError());
}

}  // namespace spmm
