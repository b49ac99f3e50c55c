// run_csrmm <graph> <dim> <impl> <transposeB>
// Reference CLI of run_csrmm.cu:46-171 on the HIP engine. Reads
// tmp/<graph>_indptr.txt / _indices.txt, values 1.0, B = randomDenseMatrix
// (mt19937_64 seeded 1234), times 10 epochs with events on stream 0 and
// prints the reference's lines. impl: gespmm (gespmm_csrmm<float>),
// cusparseScsrmm (col-major B and C), cusparseScsrmm2 (transposeB picks the
// B layout, col-major C) — all served by libspmm_hip.so.
#include <cassert>
#include <iostream>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 5) {
    printf("usage: %s <graph> <dim> <gespmm|cusparseScsrmm|cusparseScsrmm2> <transposeB>\n",
           argv[0]);
    return 1;
  }
  std::string prefix = "tmp/" + std::string(argv[1]);
  int dim = std::stoi(argv[2]);
  std::string impl(argv[3]);
  int transposeB = std::stoi(argv[4]);
  printf("graph = %s dim = %d csrmmImpl = %s transposeB = %d\n", argv[1], dim, impl.c_str(),
         transposeB);
  printf("load CSR matrix...\n");
  std::vector<int> rp, ci;
  load_csr_or_die(prefix, rp, ci);
  const int n = (int)rp.size() - 1;
  const int nnz = (int)ci.size();
  std::cout << "n=" << n << " nnz=" << nnz << std::endl;
  std::vector<float> val(nnz, 1.0f);
  std::vector<float> y = random_dense(n, dim);

  printf("gpu memory malloc and memcpy...\n");
  DeviceArena mem;
  int* d_rp = mem.upload(rp.data(), rp.size());
  int* d_ci = mem.upload(ci.data(), ci.size());
  float* d_val = mem.upload(val.data(), val.size());
  float* d_y = mem.upload(y.data(), y.size());
  float* d_z = mem.alloc<float>((size_t)n * dim);
  HANDLE_ERROR(hipMemset(d_z, 0, (size_t)n * dim * sizeof(float)));

  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t descr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&descr));
  const float alpha = 1.f, beta = 0.f;
  const int ldb = transposeB == 0 ? n : dim;
  // For the cuSPARSE-shaped impls a column-major B of the same values is
  // needed (transposeB == 0); gespmm always reads B row-major.
  float* d_yc = nullptr;
  if (impl != "gespmm" && transposeB == 0) {
    std::vector<float> yc((size_t)n * dim);
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < dim; ++c) yc[(size_t)c * n + r] = y[(size_t)r * dim + c];
    d_yc = mem.upload(yc.data(), yc.size());
  }
  printf("csrmm...\n");
  const int epoch = 10;
  float total = 0.f;
  EventTimer tm;
  for (int i = 0; i < epoch; ++i) {
    tm.start();
    if (impl == "gespmm") {
      gespmm_csrmm<float>(n, dim, d_rp, d_ci, d_val, d_y, d_z);
    } else if (impl == "cusparseScsrmm") {
      assert(transposeB == 0);
      HANDLE_SPMM_ERROR(spmm_scsrmm(handle, SPMM_OPERATION_NON_TRANSPOSE, n, dim, n, nnz, &alpha,
                                    descr, d_val, d_rp, d_ci, d_yc, ldb, &beta, d_z, n));
    } else if (impl == "cusparseScsrmm2") {
      HANDLE_SPMM_ERROR(spmm_scsrmm2(
          handle, SPMM_OPERATION_NON_TRANSPOSE,
          transposeB ? SPMM_OPERATION_TRANSPOSE : SPMM_OPERATION_NON_TRANSPOSE, n, dim, n, nnz,
          &alpha, descr, d_val, d_rp, d_ci, transposeB ? d_y : d_yc, ldb, &beta, d_z, n));
    } else {
      printf("unknown impl %s\n", impl.c_str());
      return 1;
    }
    const float t = tm.stop_ms();
    HANDLE_ERROR(hipGetLastError());
    printf("csrmm cost time:  %3.10f ms \n", t);
    total += t;
  }
  const float avg = total / epoch;
  printf("average csrmm cost time: %3.10f ms\n", avg);
  printf("GFLOP/s (2*nnz*dim/t): %6.3f\n", 2.0 * nnz * dim / (avg * 1e6));
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
