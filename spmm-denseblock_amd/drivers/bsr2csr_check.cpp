// bsr2csr_check <p> <blockDim>
// The reference's differential program bsr2csr.cu (:90-311) on the HIP
// engine: m = n = 4096, dim = 100; randomBSRMatrix(m/bs, n/bs, bs, p) then
// randomDenseMatrix(n, dim) from the seeded mt19937_64 (bit-exact with the
// reference's load_data.cc); device bsr2csr (cusparseSbsr2csr shape,
// explicit zeros kept: nnz = nnzb * bs^2, :177-188); z1 = csrmm
// (cusparseScsrmm, B and C col-major, ldb = n, ldc = m, :248-250) and
// z2 = bsrmm (cusparseSbsrmm ROW, transB = N, :228-231); "same result" when
// no |z1 - z2| exceeds 0.05 (:296-310). SPMM_DRIVER_DUMP: z2, row-major.
#include <cmath>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 3) {
    printf("usage: %s <p> <blockDim>\n", argv[0]);
    return 1;
  }
  const float p = std::stof(argv[1]);
  const int bs = (int)std::stof(argv[2]);
  printf("p = %f blockDim = %d\n", p, bs);
  const int m = 4096, n = 4096, dim = 100;
  const int mb = m / bs, nb = n / bs;
  std::vector<int> brp(mb + 1);
  int* c = nullptr;
  float* v = nullptr;
  const int nnzb = (int)spmm_host_random_bsr(mb, nb, bs, p, -1.f, 1.f, brp.data(), &c, &v);
  std::vector<int> bci(c, c + nnzb);
  std::vector<float> bval(v, v + (size_t)nnzb * bs * bs);
  spmm_host_free(c);
  spmm_host_free(v);
  const int nnz = nnzb * bs * bs;
  std::vector<float> y = random_dense(n, dim);  // read column-major, ldb = n

  DeviceArena mem;
  int* d_brp = mem.upload(brp.data(), brp.size());
  int* d_bci = mem.upload(bci.data(), bci.size());
  float* d_bval = mem.upload(bval.data(), bval.size());
  float* d_y = mem.upload(y.data(), y.size());
  int* d_rp = mem.alloc<int>((size_t)mb * bs + 1);
  int* d_ci = mem.alloc<int>(nnz);
  float* d_val = mem.alloc<float>(nnz);
  float* d_z1 = mem.alloc<float>((size_t)m * dim);
  float* d_z2 = mem.alloc<float>((size_t)m * dim);
  HANDLE_ERROR(hipMemset(d_z1, 0, (size_t)m * dim * sizeof(float)));
  HANDLE_ERROR(hipMemset(d_z2, 0, (size_t)m * dim * sizeof(float)));
  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t csrDescr = nullptr, bsrDescr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&csrDescr));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&bsrDescr));
  HANDLE_SPMM_ERROR(spmm_sbsr2csr_dev(handle, SPMM_DIRECTION_ROW, mb, nb, bsrDescr, d_bval, d_brp,
                                      d_bci, bs, csrDescr, d_val, d_rp, d_ci));
  printf("nnzb = %d nnz = %d\n", nnzb, nnz);
  const float fone = 1.f, fzero = 0.f;
  EventTimer tm;
  tm.start();
  HANDLE_SPMM_ERROR(spmm_sbsrmm(handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE,
                                SPMM_OPERATION_NON_TRANSPOSE, mb, dim, nb, nnzb, &fone, bsrDescr,
                                d_bval, d_brp, d_bci, bs, d_y, n, &fzero, d_z2, m));
  printf("bsrmm cost time:  %3.10f ms \n", tm.stop_ms());
  tm.start();
  HANDLE_SPMM_ERROR(spmm_scsrmm(handle, SPMM_OPERATION_NON_TRANSPOSE, m, dim, n, nnz, &fone,
                                csrDescr, d_val, d_rp, d_ci, d_y, n, &fzero, d_z1, m));
  printf("csrmm cost time:  %3.10f ms \n", tm.stop_ms());
  std::vector<float> z1((size_t)m * dim), z2((size_t)m * dim);
  HANDLE_ERROR(hipMemcpy(z1.data(), d_z1, z1.size() * sizeof(float), hipMemcpyDeviceToHost));
  HANDLE_ERROR(hipMemcpy(z2.data(), d_z2, z2.size() * sizeof(float), hipMemcpyDeviceToHost));
  bool flag = true;
  for (int i = 0; i < m * dim; ++i) {
    const float error = std::fabs(z1[i] - z2[i]);
    if (error > 0.05f) {
      printf("inconsistent result: %d %f", i, error);
      flag = false;
      break;
    }
  }
  printf(flag ? "\nsame result\n" : "\ninconsistent result\n");
  std::vector<float> zr((size_t)m * dim);
  for (int r = 0; r < m; ++r)
    for (int k = 0; k < dim; ++k) zr[(size_t)r * dim + k] = z2[(size_t)k * m + r];
  dump_result(zr);
  spmm_destroy_mat_descr(csrDescr);
  spmm_destroy_mat_descr(bsrDescr);
  spmm_destroy(handle);
  printf("end\n");
  return flag ? 0 : 1;
}
