// driver_common.hpp — shared plumbing for the reference-compatible drivers
// (run_csrmm, run_bsrmm, test_csrmm, test_bsrmm). Same error convention as
// the reference: print "<error> in <file> at line<N>", clean up, exit(-1)
// (utility.cc:15-29, run_csrmm.cu:17-44).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "spmm_compat.hpp"
#include "spmm_hip.h"
#include "spmm_host.h"

inline bool checkError(hipError_t err, const char* file, int line) {
  if (err != hipSuccess) {
    printf("%s in %s at line%d\n", hipGetErrorString(err), file, line);
    return false;
  }
  return true;
}

inline bool checkSpmmError(spmm_status_t status, const char* file, int line) {
  if (status != SPMM_STATUS_SUCCESS) {
    printf("%s in %s at line%d\n", spmm_get_status_string(status), file, line);
    return false;
  }
  return true;
}

// Device buffers freed at exit (the reference's CLEANUP macro).
struct DeviceArena {
  std::vector<void*> ptrs;
  template <typename T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) {
      printf("hipMalloc of %zu bytes failed\n", n * sizeof(T));
      exit(-1);
    }
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  template <typename T>
  T* upload(const T* h, size_t n) {
    T* d = alloc<T>(n);
    if (n && hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) exit(-1);
    return d;
  }
  ~DeviceArena() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

#define HANDLE_ERROR(err)                     \
  if (!checkError(err, __FILE__, __LINE__)) { \
    printf("HIP ERROR\n");                    \
    exit(-1);                                 \
  }

#define HANDLE_SPMM_ERROR(err)                    \
  if (!checkSpmmError(err, __FILE__, __LINE__)) { \
    printf("SPMM ERROR\n");                       \
    exit(-1);                                     \
  }

// loadCSRFromFile (load_data.cc:143-165) with the reference's "tmp/" prefix, through the
// binary sidecar cache (<prefix>.csrbin, rewritten whenever the text is newer).
inline void load_csr_or_die(const std::string& prefix, std::vector<int>& rp,
                            std::vector<int>& ci) {
  int *r = nullptr, *c = nullptr, n = 0;
  int64_t nnz = 0;
  if (spmm_host_load_csr_cached(prefix.c_str(), &r, &c, &n, &nnz) != 0) {
    printf("cannot read %s_indptr.txt / %s_indices.txt\n", prefix.c_str(), prefix.c_str());
    exit(-1);
  }
  rp.assign(r, r + n + 1);
  ci.assign(c, c + nnz);
  spmm_host_free(r);
  spmm_host_free(c);
}

inline std::vector<float> random_dense(int64_t n, int64_t dim) {
  std::vector<float> v((size_t)(n * dim));
  spmm_host_random_array(n * dim, -1.f, 1.f, v.data());
  return v;
}

struct EventTimer {
  hipEvent_t a, b;
  EventTimer() {
    HANDLE_ERROR(hipEventCreate(&a));
    HANDLE_ERROR(hipEventCreate(&b));
  }
  void start() { HANDLE_ERROR(hipEventRecord(a, 0)); }
  float stop_ms() {
    float t = 0.f;
    HANDLE_ERROR(hipEventRecord(b, 0));
    HANDLE_ERROR(hipEventSynchronize(b));
    HANDLE_ERROR(hipEventElapsedTime(&t, a, b));
    return t;
  }
  ~EventTimer() {
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
};

// SPMM_DRIVER_DUMP=<path>: write the result C (row-major rows x dim float32)
// so a test can check it element by element against the oracle. Not in the
// reference (whose drivers print timings only); off unless set.
inline void dump_result(const std::vector<float>& z) {
  const char* path = getenv("SPMM_DRIVER_DUMP");
  if (!path || !*path) return;
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(z.data()), (std::streamsize)(z.size() * sizeof(float)));
  if (!f) {
    printf("cannot write %s\n", path);
    exit(-1);
  }
}
