// run_bsrmm <graph> <blockDim> <dim> <rocsparse|cusparse>
// Reference CLI of run_bsrmm.cu:46-186 on the HIP engine: values 1.0,
// csr2bsr on the HOST (north_star: conversion stays CPU-side; the reference
// used cusparseXcsr2bsrNnz + cusparseScsr2bsr on the GPU, run_bsrmm.cu:116-142),
// y = randomDenseMatrix(nb*bs, dim) read column-major (ldb = nb*bs),
// alpha = beta = 1 onto zeroed z, one timed call.
#include <iostream>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 5) {
    printf("usage: %s <graph> <blockDim> <dim> <rocsparse|cusparse>\n", argv[0]);
    return 1;
  }
  std::string prefix = "tmp/" + std::string(argv[1]);
  std::cout << prefix << std::endl;
  const int bs = std::stoi(argv[2]);
  const int dim = std::stoi(argv[3]);
  std::string impl(argv[4]);
  printf("load CSR matrix...\n");
  std::vector<int> rp, ci;
  load_csr_or_die(prefix, rp, ci);
  const int n = (int)rp.size() - 1;
  const int nnz = (int)ci.size();
  std::cout << "n=" << n << " nnz=" << nnz << std::endl;
  std::vector<float> val(nnz, 1.0f);
  const int nb = (n + bs - 1) / bs;
  std::vector<float> y = random_dense((int64_t)nb * bs, dim);

  // Host csr2bsr, two-phase like cusparseXcsr2bsrNnz / cusparseScsr2bsr.
  std::vector<int> brp(nb + 1);
  int nnzb = 0;
  HANDLE_SPMM_ERROR(spmm_xcsr2bsr_nnz(SPMM_DIRECTION_ROW, n, n, rp.data(), ci.data(), bs,
                                      brp.data(), &nnzb));
  const long long numVal = (long long)nnzb * bs * bs * (long long)sizeof(float);
  printf("numVal = %lld\n", numVal);
  std::vector<int> bci(nnzb);
  std::vector<float> bval((size_t)nnzb * bs * bs);
  HANDLE_SPMM_ERROR(spmm_scsr2bsr(SPMM_DIRECTION_ROW, n, n, val.data(), rp.data(), ci.data(), bs,
                                  brp.data(), bval.data(), bci.data()));
  printf("density:  %3.10f \n", (1.0 * nnzb) / ((nb * 1.0) * (nb * 1.0)));

  printf("gpu memory malloc and memcpy...\n");
  DeviceArena mem;
  int* d_brp = mem.upload(brp.data(), brp.size());
  int* d_bci = mem.upload(bci.data(), bci.size());
  float* d_bval = mem.upload(bval.data(), bval.size());
  float* d_y = mem.upload(y.data(), y.size());
  float* d_z = mem.alloc<float>((size_t)nb * bs * dim);
  HANDLE_ERROR(hipMemset(d_z, 0, (size_t)nb * bs * dim * sizeof(float)));
  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t descr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&descr));
  const float alpha = 1.f, beta = 1.f;
  printf("bsrmm...\n");
  EventTimer tm;
  tm.start();
  if (impl == "rocsparse") {
    HANDLE_SPMM_ERROR(rocsparse_bsrmm_template<float>(
        handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE, SPMM_OPERATION_NON_TRANSPOSE,
        nb, dim, nb, nnzb, alpha, descr, d_bval, d_brp, d_bci, bs, d_y, nb * bs, beta, d_z,
        nb * bs));
  } else if (impl == "cusparse") {
    HANDLE_SPMM_ERROR(spmm_sbsrmm(handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE,
                                  SPMM_OPERATION_NON_TRANSPOSE, nb, dim, nb, nnzb, &alpha, descr,
                                  d_bval, d_brp, d_bci, bs, d_y, nb * bs, &beta, d_z, nb * bs));
  } else {
    printf("unknown impl %s\n", impl.c_str());
    return 1;
  }
  const float t = tm.stop_ms();
  printf("bsrmm cost time:  %3.10f ms \n", t);
  printf("useful GFLOP/s (2*nnz*dim/t): %6.3f  MFMA-executed GFLOP/s (2*nnzb*bs^2*dim/t): %6.3f\n",
         2.0 * nnz * dim / (t * 1e6), 2.0 * nnzb * bs * (double)bs * dim / (t * 1e6));
  {  // z is column-major (ldc = nb*bs): rows 0 .. n-1, row-major for the dump
    std::vector<float> zc((size_t)nb * bs * dim), z((size_t)n * dim);
    HANDLE_ERROR(hipMemcpy(zc.data(), d_z, zc.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < dim; ++c) z[(size_t)r * dim + c] = zc[(size_t)c * nb * bs + r];
    dump_result(z);
  }
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
