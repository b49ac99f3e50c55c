// test_bsrmm <p> <blockDim> <dim> <rocsparse|cusparse> <transposeB>
// Reference CLI of test_bsrmm.cu:46-181: m = n = 2<<16, random BSR pattern
// from tmp/bsr_<mb>_<nb>_<bs>_<nnzb> (values redrawn) or generated with
// randomBSRMatrix and dumped, one timed call, prints "GFLOPs" as the
// reference (nnzb*bs^2*dim/t).
#include <sys/stat.h>

#include <cassert>
#include <sstream>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 6) {
    printf("usage: %s <p> <blockDim> <dim> <rocsparse|cusparse> <transposeB>\n", argv[0]);
    return 1;
  }
  const float p = std::stof(argv[1]);
  const int bs = std::stoi(argv[2]);
  const int dim = std::stoi(argv[3]);
  std::string impl(argv[4]);
  const int transposeB = std::stoi(argv[5]);
  printf("p = %f blockDim = %d dim = %d bsrmmImpl = %s transposeB = %d\n", p, bs, dim,
         impl.c_str(), transposeB);
  const int m = 2 << 16, n = m;
  const int mb = (m + bs - 1) / bs, nb = (n + bs - 1) / bs;
  assert(mb * bs == m && nb * bs == n);
  std::stringstream ss;
  ss << "tmp/bsr_" << mb << "_" << nb << "_" << bs << "_" << (int)(mb * (nb * p));
  const std::string name = ss.str();
  std::vector<int> rp(mb + 1), ci;
  std::vector<float> val;
  struct stat st;
  if (stat((name + "_indptr.txt").c_str(), &st) == 0) {
    load_csr_or_die(name, rp, ci);
    val.resize(ci.size() * bs * bs);
    spmm_host_random_array((int64_t)val.size(), -1.f, 1.f, val.data());
  } else {
    printf("generate random BSR matrix\n");
    int* c = nullptr;
    float* v = nullptr;
    const int64_t nnzb = spmm_host_random_bsr(mb, nb, bs, p, -1.f, 1.f, rp.data(), &c, &v);
    ci.assign(c, c + nnzb);
    val.assign(v, v + nnzb * bs * bs);
    spmm_host_free(c);
    spmm_host_free(v);
    mkdir("tmp", 0755);
    spmm_host_dump_csr(name.c_str(), mb, nnzb, rp.data(), ci.data());
  }
  const int nnzb = (int)ci.size();
  printf("nnzb = %d mb = %d nb = %d\n", nnzb, mb, nb);
  printf("density of BSR matrix is %f\n", (nnzb * 1.0) / ((mb * 1.0) * (nb * 1.0)));
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
  const spmm_operation_t tB = transposeB ? SPMM_OPERATION_TRANSPOSE : SPMM_OPERATION_NON_TRANSPOSE;
  const int ldb = transposeB ? dim : n;
  const float fone = 1.f, fzero = 0.f;
  EventTimer tm;
  tm.start();
  if (impl == "rocsparse") {
    HANDLE_SPMM_ERROR(rocsparse_bsrmm_template<float>(
        handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE, tB, mb, dim, nb, nnzb, fone,
        descr, d_val, d_rp, d_ci, bs, d_y, ldb, fzero, d_z, m));
  } else if (impl == "cusparse") {
    HANDLE_SPMM_ERROR(spmm_sbsrmm(handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE, tB, mb,
                                  dim, nb, nnzb, &fone, descr, d_val, d_rp, d_ci, bs, d_y, ldb,
                                  &fzero, d_z, m));
  } else {
    printf("unknown impl %s\n", impl.c_str());
    return 1;
  }
  const float t = tm.stop_ms();
  printf("bsrmm cost time: %6.10f ms\nGFLOPs: %6.10f\n", t,
         (nnzb / 1.0e6) * (bs * bs * dim) / t);
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
