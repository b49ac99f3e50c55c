// test_csrmm <p> <dim> <gespmm|cusparse>
// Reference CLI of test_csrmm.cu:46-153: m = n = 2<<16 synthetic CSR from
// readAndFillCSRMatrix (tmp/csr__<m>_<n>_<nnz> pattern, values redrawn), or
// generated with randomCSRMatrix and dumped there when the file is missing.
// One timed call; prints the reference's "GFLOPs" (= nnz*dim/t, i.e. half
// of 2*nnz*dim/t) plus the 2*nnz*dim/t figure.
#include <sys/stat.h>

#include <sstream>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 4) {
    printf("usage: %s <p> <dim> <gespmm|cusparse>\n", argv[0]);
    return 1;
  }
  const float p = std::stof(argv[1]);
  const int dim = std::stoi(argv[2]);
  std::string impl(argv[3]);
  printf("p = %f dim = %d csrmmImpl = %s\n", p, dim, impl.c_str());
  const int m = 2 << 16, n = m;
  std::stringstream ss;
  ss << "tmp/csr_" << "_" << m << "_" << n << "_" << (int)(m * (n * p));  // load_data.cc:14-20
  const std::string name = ss.str();
  std::vector<int> rp(m + 1), ci;
  std::vector<float> val;
  struct stat st;
  if (stat((name + "_indptr.txt").c_str(), &st) == 0) {
    load_csr_or_die(name, rp, ci);
    val.resize(ci.size());
    spmm_host_random_array((int64_t)ci.size(), -1.f, 1.f, val.data());
  } else {
    printf("generate random CSR matrix\n");
    int* c = nullptr;
    float* v = nullptr;
    const int64_t nnz = spmm_host_random_csr(m, n, p, -1.f, 1.f, rp.data(), &c, &v);
    ci.assign(c, c + nnz);
    val.assign(v, v + nnz);
    spmm_host_free(c);
    spmm_host_free(v);
    mkdir("tmp", 0755);
    spmm_host_dump_csr(name.c_str(), m, nnz, rp.data(), ci.data());
  }
  const int nnz = (int)ci.size();
  printf("density of CSR matrix is %f\n", ((nnz * 1.0) / m) / n);
  printf("prepare y and z...\n");
  std::vector<float> y = random_dense(n, dim);
  DeviceArena mem;
  int* d_rp = mem.upload(rp.data(), rp.size());
  int* d_ci = mem.upload(ci.data(), ci.size());
  float* d_val = mem.upload(val.data(), val.size());
  float* d_y = mem.upload(y.data(), y.size());
  float* d_z = mem.alloc<float>((size_t)m * dim);
  HANDLE_ERROR(hipMemset(d_z, 0, (size_t)m * dim * sizeof(float)));
  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t descr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&descr));
  const float fone = 1.f, fzero = 0.f;
  EventTimer tm;
  tm.start();
  if (impl == "gespmm") {
    gespmm_csrmm<float>(m, dim, d_rp, d_ci, d_val, d_y, d_z);
  } else if (impl == "cusparse") {
    // cusparseScsrmm2(N, T): B row-major (ldb = dim), C column-major (ldc = m)
    HANDLE_SPMM_ERROR(spmm_scsrmm2(handle, SPMM_OPERATION_NON_TRANSPOSE, SPMM_OPERATION_TRANSPOSE,
                                   m, dim, n, nnz, &fone, descr, d_val, d_rp, d_ci, d_y, dim,
                                   &fzero, d_z, m));
  } else {
    printf("unknown impl %s\n", impl.c_str());
    return 1;
  }
  const float t = tm.stop_ms();
  HANDLE_ERROR(hipGetLastError());
  printf("csrmm cost time: %6.10f ms\nGFLOPs: %6.10f\n", t, (nnz / 1.0e6) * dim / t);
  printf("GFLOP/s (2*nnz*dim/t): %6.3f\n", 2.0 * nnz * dim / (t * 1e6));
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
