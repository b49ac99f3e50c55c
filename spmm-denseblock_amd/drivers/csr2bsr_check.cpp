// csr2bsr_check <p>
// The reference's differential program csr2bsr.cu (:87-311) on the HIP
// engine: m = 1000, n = 1200, blockDim = 2, dim = 100;
// randomCSRMatrix(m, n, p) then randomDenseMatrix(n, dim) from the seeded
// mt19937_64 (bit-exact with the reference's load_data.cc); device csr2bsr
// (cusparseXcsr2bsrNnz + cusparseScsr2bsr shapes, :163-192); z1 = csrmm
// (cusparseScsrmm: B and C col-major, ldb = n, ldc = m, :232-234) and
// z2 = bsrmm (cusparseSbsrmm ROW, transB = N, ldb = n, ldc = m, :251-254);
// "same result" when no |z1 - z2| exceeds 0.01 (:297-311). With
// SPMM_DRIVER_DUMP set, z2 is written row-major for the oracle check.
#include <cmath>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 2) {
    printf("usage: %s <p>\n", argv[0]);
    return 1;
  }
  const float p = std::stof(argv[1]);
  printf("%f\n", p);
  const int m = 1000, n = 1200, bs = 2, dim = 100;
  const int mb = (m + bs - 1) / bs, nb = (n + bs - 1) / bs;
  std::vector<int> rp(m + 1);
  int* c = nullptr;
  float* v = nullptr;
  const int nnz = (int)spmm_host_random_csr(m, n, p, -1.f, 1.f, rp.data(), &c, &v);
  std::vector<int> ci(c, c + nnz);
  std::vector<float> val(v, v + nnz);
  spmm_host_free(c);
  spmm_host_free(v);
  std::vector<float> y = random_dense(n, dim);  // read column-major, ldb = n

  DeviceArena mem;
  int* d_rp = mem.upload(rp.data(), rp.size());
  int* d_ci = mem.upload(ci.data(), ci.size());
  float* d_val = mem.upload(val.data(), val.size());
  float* d_y = mem.upload(y.data(), y.size());
  float* d_z1 = mem.alloc<float>((size_t)m * dim);
  float* d_z2 = mem.alloc<float>((size_t)m * dim);
  HANDLE_ERROR(hipMemset(d_z1, 0, (size_t)m * dim * sizeof(float)));
  HANDLE_ERROR(hipMemset(d_z2, 0, (size_t)m * dim * sizeof(float)));
  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t csrDescr = nullptr, bsrDescr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&csrDescr));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&bsrDescr));
  int* d_brp = mem.alloc<int>(mb + 1);
  int nnzb = 0;
  HANDLE_SPMM_ERROR(spmm_xcsr2bsr_nnz_dev(handle, SPMM_DIRECTION_ROW, m, n, csrDescr, d_rp, d_ci,
                                          bs, bsrDescr, d_brp, &nnzb));
  int* d_bci = mem.alloc<int>(nnzb);
  float* d_bval = mem.alloc<float>((size_t)nnzb * bs * bs);
  HANDLE_SPMM_ERROR(spmm_scsr2bsr_dev(handle, SPMM_DIRECTION_ROW, m, n, csrDescr, d_val, d_rp,
                                      d_ci, bs, bsrDescr, d_bval, d_brp, d_bci));
  const float fone = 1.f, fzero = 0.f;
  EventTimer tm;
  tm.start();
  HANDLE_SPMM_ERROR(spmm_scsrmm(handle, SPMM_OPERATION_NON_TRANSPOSE, m, dim, n, nnz, &fone,
                                csrDescr, d_val, d_rp, d_ci, d_y, n, &fzero, d_z1, m));
  printf("csrmm cost time:  %3.10f ms \n", tm.stop_ms());
  tm.start();
  HANDLE_SPMM_ERROR(spmm_sbsrmm(handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE,
                                SPMM_OPERATION_NON_TRANSPOSE, mb, dim, nb, nnzb, &fone, bsrDescr,
                                d_bval, d_brp, d_bci, bs, d_y, n, &fzero, d_z2, m));
  printf("bsrmm cost time:  %3.10f ms \n", tm.stop_ms());
  std::vector<float> z1((size_t)m * dim), z2((size_t)m * dim);
  HANDLE_ERROR(hipMemcpy(z1.data(), d_z1, z1.size() * sizeof(float), hipMemcpyDeviceToHost));
  HANDLE_ERROR(hipMemcpy(z2.data(), d_z2, z2.size() * sizeof(float), hipMemcpyDeviceToHost));
  bool flag = true;
  for (int i = 0; i < m * dim; ++i) {
    const float error = std::fabs(z1[i] - z2[i]);
    if (error > 0.01f) {
      printf("inconsistent result: %d %f", i, error);
      flag = false;
      break;
    }
  }
  printf(flag ? "\nsame result\n" : "\ninconsistent result\n");
  std::vector<float> zr((size_t)m * dim);  // col-major (ldc = m) -> row-major
  for (int r = 0; r < m; ++r)
    for (int k = 0; k < dim; ++k) zr[(size_t)r * dim + k] = z2[(size_t)k * m + r];
  dump_result(zr);
  spmm_destroy_mat_descr(csrDescr);
  spmm_destroy_mat_descr(bsrDescr);
  spmm_destroy(handle);
  printf("end\n");
  return flag ? 0 : 1;
}
