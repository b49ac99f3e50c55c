// Practical HBM ceiling on the box: a streaming read (dwordx4 per lane,
// grid-stride, non-temporal) and a streaming copy over 4 GiB, timed with HIP
// events. Context for the CSR kernel's fabric rate: the spec
// peak is 8 TB/s; this is what plain streams reach.
//   hipcc -O3 --offload-arch=gfx950 tools/hbm_peak.hip -o /tmp/hbm_peak && /tmp/hbm_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void read_kernel(const f32x4* __restrict__ x, size_t n,
                                                   float* __restrict__ out) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = i + u * stride < n ? __builtin_nontemporal_load(x + i + u * stride) : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[0] = s;  // keeps the loads live
}

__global__ __launch_bounds__(256) void copy_kernel(const f32x4* __restrict__ x, f32x4* __restrict__ y,
                                                   size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  const size_t bytes = (size_t)4 << 30, n = bytes / 16;
  f32x4 *x, *y;
  float* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int blocks_per_cu : {4, 8, 16, 32, 64}) {
    const int grid = 256 * blocks_per_cu;
    float best_r = 1e30f, best_r8 = 1e30f, best_c = 1e30f;
    for (int rep = 0; rep < 12; ++rep) {
      float ms;
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(read_kernel<8>, dim3(grid), dim3(256), 0, 0, x, n, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep >= 2 && ms < best_r8) best_r8 = ms;
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(read_kernel<4>, dim3(grid), dim3(256), 0, 0, x, n, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep >= 2 && ms < best_r) best_r = ms;
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, x, y, n);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep >= 2 && ms < best_c) best_c = ms;
    }
    printf("{\"workgroups_per_cu\": %d, \"read_GBps\": %.0f, \"read8_GBps\": %.0f, \"copy_GBps\": %.0f}\n",
           blocks_per_cu, bytes / (best_r * 1e-3) / 1e9, bytes / (best_r8 * 1e-3) / 1e9,
           2.0 * bytes / (best_c * 1e-3) / 1e9);
  }
  return 0;
}
