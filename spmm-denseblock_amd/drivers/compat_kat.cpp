// compat_kat <float|double>  < problems.txt
// The reference's C++ call shapes, compiled against include/spmm_compat.hpp:
// gespmm_csrmm<T> (gespmm_csrmm.h:422-426) and rocsparse_bsrmm_template<T>
// (rocsparse_bsrmm.h:102-108), on problems read from stdin (the known-answer
// programs' data, fed by tests/test_drivers.py from tests/golden/kats.json):
//   csr <m> <k> <n> <nnz>  rowptr[m+1] colind[nnz] val[nnz] B[k*n] (row-major)
//       -> gespmm_csrmm<T>, prints "C" + m*n values (row-major)
//   bsr <dir> <transB> <mb> <kb> <n> <bs> <nnzb> <ldb> <ldc> <beta>
//       rowptr[mb+1] colind[nnzb] val[nnzb*bs*bs] B[(transB ? kb*bs : n)*ldb]
//       -> rocsparse_bsrmm_template<T> (alpha 1, C zeroed, col-major ldc),
//       prints "C" + ldc*n values and the returned status
#include <iostream>
#include <string>

#include "driver_common.hpp"

template <class T>
static std::vector<T> read_vec(size_t n) {
  std::vector<T> v(n);
  for (auto& x : v) std::cin >> x;
  return v;
}

template <class T>
static void print_c(const std::vector<T>& c) {
  printf("C");
  for (T x : c) printf(" %.17g", (double)x);
  printf("\n");
}

template <class T>
static int run() {
  std::string kind;
  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t descr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&descr));
  while (std::cin >> kind) {
    DeviceArena mem;
    if (kind == "csr") {
      int m, k, n, nnz;
      std::cin >> m >> k >> n >> nnz;
      auto rp = read_vec<int>(m + 1);
      auto ci = read_vec<int>(nnz);
      auto v = read_vec<T>(nnz);
      auto B = read_vec<T>((size_t)k * n);
      int* d_rp = mem.upload(rp.data(), rp.size());
      int* d_ci = mem.upload(ci.data(), ci.size());
      T* d_v = mem.upload(v.data(), v.size());
      T* d_B = mem.upload(B.data(), B.size());
      T* d_C = mem.alloc<T>((size_t)m * n);
      gespmm_csrmm<T>(m, n, d_rp, d_ci, d_v, d_B, d_C);  // returns void, as the reference
      HANDLE_ERROR(hipDeviceSynchronize());
      std::vector<T> C((size_t)m * n);
      HANDLE_ERROR(hipMemcpy(C.data(), d_C, C.size() * sizeof(T), hipMemcpyDeviceToHost));
      print_c(C);
    } else if (kind == "bsr") {
      int dir, tb, mb, kb, n, bs, nnzb, ldb, ldc;
      double beta;
      std::cin >> dir >> tb >> mb >> kb >> n >> bs >> nnzb >> ldb >> ldc >> beta;
      auto rp = read_vec<int>(mb + 1);
      auto ci = read_vec<int>(nnzb);
      auto v = read_vec<T>((size_t)nnzb * bs * bs);
      auto B = read_vec<T>((size_t)(tb ? kb * bs : n) * ldb);
      int* d_rp = mem.upload(rp.data(), rp.size());
      int* d_ci = mem.upload(ci.data(), ci.size());
      T* d_v = mem.upload(v.data(), v.size());
      T* d_B = mem.upload(B.data(), B.size());
      T* d_C = mem.alloc<T>((size_t)ldc * n);
      HANDLE_ERROR(hipMemset(d_C, 0, (size_t)ldc * n * sizeof(T)));
      const spmm_status_t st = rocsparse_bsrmm_template<T>(
          handle, (spmm_direction_t)dir, SPMM_OPERATION_NON_TRANSPOSE,
          tb ? SPMM_OPERATION_TRANSPOSE : SPMM_OPERATION_NON_TRANSPOSE, mb, n, kb, nnzb, T(1),
          descr, d_v, d_rp, d_ci, bs, d_B, ldb, T(beta), d_C, ldc);
      HANDLE_ERROR(hipDeviceSynchronize());
      std::vector<T> C((size_t)ldc * n);
      HANDLE_ERROR(hipMemcpy(C.data(), d_C, C.size() * sizeof(T), hipMemcpyDeviceToHost));
      print_c(C);
      printf("status %s\n", spmm_get_status_string(st));
    } else {
      printf("unknown problem kind %s\n", kind.c_str());
      return 1;
    }
  }
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}

int main(int argc, char* argv[]) {
  const std::string t = argc > 1 ? argv[1] : "float";
  if (t == "float") return run<float>();
  if (t == "double") return run<double>();
  printf("usage: %s <float|double> < problems\n", argv[0]);
  return 1;
}
