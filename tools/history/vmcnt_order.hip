// Does a counted s_waitcnt vmcnt(N) order an LDS-DMA copy against a younger
// VGPR load (and the other way round)? The bs 32 CM4 kernel waited vmcnt(1)
// with four B-panel LDS-DMA copies followed by one A load to VGPRs in flight,
// and lost B rows ("the CM4 copy race"); its ISA shows that
// issue order (tests/test_isa_waits.py). This probe measures the rule on the
// hardware, one wave per workgroup, every instruction of the window in one
// asm block so the compiler adds no wait of its own:
//   mode 0  DMA(cold 1 KB) ; VGPR load(hot)  ; vmcnt(1) ; read the DMA's LDS
//   mode 1  DMA(cold)      ; DMA(hot)        ; vmcnt(1) ; read the cold DMA's LDS
//   mode 2  DMA(cold)      ; VGPR load(hot)  ; vmcnt(0) ; read   (control)
//   mode 3  VGPR load(cold); DMA(hot)        ; vmcnt(1) ; snapshot the cold VGPR
//   mode 4  VGPR load(cold); VGPR load(hot)  ; vmcnt(1) ; snapshot (control)
// "cold" = a random 1 KB piece of a 4 GiB buffer (HBM miss), "hot" = one
// L2-resident 1 KB piece. A trial fails when the older operation's data is not
// there after the wait (LDS still holds the sentinel / the VGPR still holds
// it). Prints one JSON line per mode.
//   hipcc -O3 --offload-arch=gfx950 tools/vmcnt_order.hip -o /tmp/vmcnt_order && /tmp/vmcnt_order
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned mix(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ float fill_of(size_t i) { return (float)(i % 1000003u) + 1.f; }

__global__ void fill_kernel(float* x, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    x[i] = fill_of(i);
}

template <int MODE>
__global__ __launch_bounds__(64) void probe_kernel(const float* __restrict__ cold, size_t chunks,
                                                   const float* __restrict__ hot, int iters,
                                                   unsigned seed, unsigned* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float lds[512];  // two 1 KB regions
  const int lane = threadIdx.x;
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  const unsigned lds1 = lds0 + 1024u;
  const unsigned la = lds0 + 16u * (unsigned)lane;
  const f32x4 sent4 = {-1.f, -1.f, -1.f, -1.f};
  const float sent = -1.f;
  unsigned stale = 0, wrong = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned h = mix(seed ^ (blockIdx.x * 0x9E3779B9u) ^ ((unsigned)it * 0x85EBCA6Bu));
    const size_t chunk = (size_t)h % chunks;
    const size_t e0 = (chunk * 64 + lane) * 4;  // this lane's 4 floats of the cold piece
    const float* ca = cold + e0;
    const float* ha = hot + 4 * lane;
    bool bad_stale = false, bad_wrong = false;
    if constexpr (MODE <= 2) {
      f32x4 got;
      float hv;
      if constexpr (MODE == 0 || MODE == 2) {
        asm volatile(
            "ds_write_b128 %[la], %[s4]\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "s_mov_b32 m0, %[m0v]\n\t"
            "global_load_lds_dwordx4 %[ca], off\n\t"
            "global_load_dword %[hv], %[ha], off\n\t"
            "s_waitcnt vmcnt(%[n])\n\t"
            "ds_read_b128 %[got], %[la]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)"
            : [got] "=&v"(got), [hv] "=&v"(hv)
            : [la] "v"(la), [s4] "v"(sent4), [m0v] "s"(lds0), [ca] "v"(ca), [ha] "v"(ha),
              [n] "i"(MODE == 0 ? 1 : 0)
            : "memory", "m0");
      } else {
        asm volatile(
            "ds_write_b128 %[la], %[s4]\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "s_mov_b32 m0, %[m0v]\n\t"
            "global_load_lds_dwordx4 %[ca], off\n\t"
            "s_mov_b32 m0, %[m1v]\n\t"
            "global_load_lds_dwordx4 %[ha], off\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "ds_read_b128 %[got], %[la]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)"
            : [got] "=&v"(got)
            : [la] "v"(la), [s4] "v"(sent4), [m0v] "s"(lds0), [m1v] "s"(lds1), [ca] "v"(ca),
              [ha] "v"(ha)
            : "memory", "m0");
        hv = 0.f;
      }
      asm volatile("" ::"v"(hv));
      for (int c = 0; c < 4; ++c) {
        if (got[c] == sent) bad_stale = true;
        else if (got[c] != fill_of(e0 + c)) bad_wrong = true;
      }
    } else {
      float cv, snap;
      if constexpr (MODE == 3) {
        asm volatile(
            "v_mov_b32 %[cv], %[s]\n\t"
            "global_load_dword %[cv], %[ca], off\n\t"
            "s_mov_b32 m0, %[m1v]\n\t"
            "global_load_lds_dwordx4 %[ha], off\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "v_mov_b32 %[snap], %[cv]\n\t"
            "s_waitcnt vmcnt(0)"
            : [cv] "=&v"(cv), [snap] "=&v"(snap)
            : [s] "v"(sent), [m1v] "s"(lds1), [ca] "v"(ca), [ha] "v"(ha)
            : "memory", "m0");
      } else {
        float hv;
        asm volatile(
            "v_mov_b32 %[cv], %[s]\n\t"
            "global_load_dword %[cv], %[ca], off\n\t"
            "global_load_dword %[hv], %[ha], off\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "v_mov_b32 %[snap], %[cv]\n\t"
            "s_waitcnt vmcnt(0)"
            : [cv] "=&v"(cv), [snap] "=&v"(snap), [hv] "=&v"(hv)
            : [s] "v"(sent), [ca] "v"(ca), [ha] "v"(ha)
            : "memory");
        asm volatile("" ::"v"(hv));
      }
      asm volatile("" ::"v"(cv));
      if (snap == sent) bad_stale = true;
      else if (snap != fill_of(e0)) bad_wrong = true;
    }
    stale += bad_stale;
    wrong += bad_wrong;
  }
  // per-lane counts, vector stores
  out[2 * ((size_t)blockIdx.x * 64 + lane)] = stale;
  out[2 * ((size_t)blockIdx.x * 64 + lane) + 1] = wrong;
}

// Cross-wave forms (4 waves per workgroup, the CM4 situation): every wave
// copies its own region(s) by LDS-DMA, issues one younger operation, waits
// vmcnt(N), then s_barrier, and reads the NEXT wave's region(s).
//   mode 5  1 DMA(cold) ; VGPR load(hot)  ; vmcnt(1) ; barrier ; read neighbour
//   mode 6  1 DMA(cold) ; DMA(hot)        ; vmcnt(1) ; barrier ; read neighbour
//   mode 7  1 DMA(cold) ; VGPR load(hot)  ; vmcnt(0) ; barrier ; read neighbour (control)
//   mode 8  4 DMA(cold) ; VGPR load(cold) ; vmcnt(1) ; barrier ; read neighbour's 4
//   mode 9  4 DMA(cold) ; VGPR load(cold) ; vmcnt(0) ; barrier ; read neighbour's 4 (control)
#define DMA1(I) "s_mov_b32 m0, %[m" #I "]\n\tglobal_load_lds_dwordx4 %[c" #I "], off\n\t"
template <int MODE>
__global__ __launch_bounds__(256) void probe_xwave_kernel(const float* __restrict__ cold,
                                                          size_t chunks,
                                                          const float* __restrict__ hot, int iters,
                                                          unsigned seed,
                                                          unsigned* __restrict__ out) {
  constexpr int ND = MODE >= 8 ? 4 : 1;
  __shared__ __attribute__((aligned(16))) float lds[4 * 4 * 256 + 4 * 256];  // 4 waves x 4 KB + scratch
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned base = (unsigned)(uintptr_t)lds;
  const unsigned own = base + 4096u * (unsigned)wv;
  const unsigned nbr = base + 4096u * (unsigned)((wv + 1) & 3);
  const unsigned scratch = base + 16384u + 1024u * (unsigned)wv;
  const f32x4 sent4 = {-1.f, -1.f, -1.f, -1.f};
  unsigned stale = 0, wrong = 0;
  for (int it = 0; it < iters; ++it) {
    size_t e[4];
    const float* ca[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const unsigned h = mix(seed ^ (blockIdx.x * 0x9E3779B9u) ^ ((unsigned)it * 0x85EBCA6Bu) ^
                             ((unsigned)(4 * wv + d) * 0xC2B2AE35u));
      e[d] = (((size_t)h % chunks) * 64 + lane) * 4;
      ca[d] = cold + e[d];
    }
    const unsigned hy = mix(seed * 31u + blockIdx.x * 977u + (unsigned)it * 13u + (unsigned)wv);
    const float* ya = MODE >= 8 ? cold + (((size_t)hy % chunks) * 64 + lane) * 4 : hot + 4 * lane;
    // sentinel into own regions, everyone's sentinel in before any copy
    for (int d = 0; d < ND; ++d)
      asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(own + 1024u * d + 16u * lane),
                   "v"(sent4) : "memory");
    __syncthreads();
    float yv = 0.f;
    if constexpr (MODE == 5 || MODE == 7) {
      asm volatile(DMA1(0) "global_load_dword %[yv], %[ya], off\n\t"
                   "s_waitcnt vmcnt(%[n])\n\ts_barrier"
                   : [yv] "=&v"(yv)
                   : [m0] "s"(own), [c0] "v"(ca[0]), [ya] "v"(ya), [n] "i"(MODE == 5 ? 1 : 0)
                   : "memory", "m0");
    } else if constexpr (MODE == 6) {
      asm volatile(DMA1(0) "s_mov_b32 m0, %[ms]\n\tglobal_load_lds_dwordx4 %[ya], off\n\t"
                   "s_waitcnt vmcnt(1)\n\ts_barrier"
                   :
                   : [m0] "s"(own), [c0] "v"(ca[0]), [ms] "s"(scratch), [ya] "v"(ya)
                   : "memory", "m0");
    } else {
      asm volatile(DMA1(0) DMA1(1) DMA1(2) DMA1(3) "global_load_dword %[yv], %[ya], off\n\t"
                   "s_waitcnt vmcnt(%[n])\n\ts_barrier"
                   : [yv] "=&v"(yv)
                   : [m0] "s"(own), [m1] "s"(own + 1024u), [m2] "s"(own + 2048u),
                     [m3] "s"(own + 3072u), [c0] "v"(ca[0]), [c1] "v"(ca[1]), [c2] "v"(ca[2]),
                     [c3] "v"(ca[3]), [ya] "v"(ya), [n] "i"(MODE == 8 ? 1 : 0)
                   : "memory", "m0");
    }
    bool bs = false, bw = false;
    for (int d = 0; d < ND; ++d) {
      f32x4 got;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(got) : "v"(nbr + 1024u * d + 16u * lane) : "memory");
      // the neighbour's expected values: recompute its random pieces
      const unsigned w2 = (wv + 1) & 3;
      const unsigned h = mix(seed ^ (blockIdx.x * 0x9E3779B9u) ^ ((unsigned)it * 0x85EBCA6Bu) ^
                             ((unsigned)(4 * w2 + d) * 0xC2B2AE35u));
      const size_t e2 = (((size_t)h % chunks) * 64 + lane) * 4;
      for (int c = 0; c < 4; ++c) {
        if (got[c] == -1.f) bs = true;
        else if (got[c] != fill_of(e2 + c)) bw = true;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::"v"(yv));
    stale += bs;
    wrong += bw;
    __syncthreads();  // every read done before the next sentinel
  }
  out[2 * ((size_t)blockIdx.x * 256 + threadIdx.x)] = stale;
  out[2 * ((size_t)blockIdx.x * 256 + threadIdx.x) + 1] = wrong;
}

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

template <int MODE>
static int run(const float* cold, size_t chunks, const float* hot, unsigned* out, int grid,
               int iters, int reps) {
  unsigned long long stale = 0, wrong = 0, trials = 0;
  std::vector<unsigned> h((size_t)grid * 64 * 2);
  for (int r = 0; r < reps; ++r) {
    probe_kernel<MODE><<<grid, 64>>>(cold, chunks, hot, iters, 1234u + 77u * r, out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h.size(); i += 2) { stale += h[i]; wrong += h[i + 1]; }
    trials += (unsigned long long)grid * 64 * iters;
  }
  static const char* what[] = {
      "dma(cold); vgpr_load(hot); vmcnt(1) -> dma landed?",
      "dma(cold); dma(hot); vmcnt(1) -> first dma landed?",
      "dma(cold); vgpr_load(hot); vmcnt(0) -> dma landed? (control)",
      "vgpr_load(cold); dma(hot); vmcnt(1) -> vgpr load landed?",
      "vgpr_load(cold); vgpr_load(hot); vmcnt(1) -> first load landed? (control)"};
  printf("{\"mode\": %d, \"window\": \"%s\", \"lane_trials\": %llu, \"stale\": %llu, "
         "\"wrong_value\": %llu}\n",
         MODE, what[MODE], trials, stale, wrong);
  return 0;
}

template <int MODE>
static int run_x(const float* cold, size_t chunks, const float* hot, unsigned* out, int grid,
                 int iters, int reps) {
  unsigned long long stale = 0, wrong = 0, trials = 0;
  std::vector<unsigned> h((size_t)grid * 256 * 2);
  for (int r = 0; r < reps; ++r) {
    probe_xwave_kernel<MODE><<<grid, 256>>>(cold, chunks, hot, iters, 4321u + 77u * r, out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h.size(); i += 2) { stale += h[i]; wrong += h[i + 1]; }
    trials += (unsigned long long)grid * 256 * iters;
  }
  static const char* what[] = {
      "1 dma(cold); vgpr_load(hot); vmcnt(1); barrier -> neighbour wave's dma landed?",
      "1 dma(cold); dma(hot); vmcnt(1); barrier -> neighbour wave's first dma landed?",
      "1 dma(cold); vgpr_load(hot); vmcnt(0); barrier -> neighbour wave's dma landed? (control)",
      "4 dma(cold); vgpr_load(cold); vmcnt(1); barrier -> neighbour wave's 4 dmas landed? (CM4 window)",
      "4 dma(cold); vgpr_load(cold); vmcnt(0); barrier -> neighbour wave's 4 dmas landed? (control)"};
  printf("{\"mode\": %d, \"window\": \"%s\", \"lane_trials\": %llu, \"stale\": %llu, "
         "\"wrong_value\": %llu}\n",
         MODE, what[MODE - 5], trials, stale, wrong);
  return 0;
}

int main() {
  const size_t bytes = (size_t)4 << 30, n = bytes / 4, chunks = bytes / 1024;
  float *cold, *hot;
  unsigned* out;
  const int grid = 4096, iters = 128, reps = 4;
  CK(hipMalloc(&cold, bytes));
  CK(hipMalloc(&hot, 1024));
  CK(hipMalloc(&out, (size_t)grid * 64 * 2 * 4));
  fill_kernel<<<4096, 256>>>(cold, n);
  fill_kernel<<<1, 256>>>(hot, 256);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  if (run<0>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run<1>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run<2>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run<3>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run<4>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  CK(hipFree(out));
  CK(hipMalloc(&out, (size_t)grid * 256 * 2 * 4));
  if (run_x<5>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run_x<6>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run_x<7>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run_x<8>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  if (run_x<9>(cold, chunks, hot, out, grid, iters, reps)) return 1;
  CK(hipFree(cold));
  CK(hipFree(hot));
  CK(hipFree(out));
  return 0;
}
