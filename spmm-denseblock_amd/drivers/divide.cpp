// divide <graph> <bsize> <dim> <rocsparse|cusparse|hybrid> <transposeB 0|1> <density>
// Reference CLI and lines of divide.cu:195-378 on the HIP engine: the graph's
// CSR (unit values) is split by divide_matrix (spmm_divide_nnz /
// spmm_sdivide, bit-exact with divide.cu:52-127) into dense blocks of fill >=
// density and a CSR remainder; y = randomDenseMatrix(n1, dim) (n1 = nb *
// bsize), z zeroed, alpha = beta = 1, and the two products accumulate into
// the column-major z (ldc = n1), each timed with events on stream 0:
//   csrmm2 (transA = N, transB = N: y column-major, ldb = n; T: y row-major,
//   ldb = dim), then bsrmm (rocsparse_bsrmm_template<float> or cusparseSbsrmm
//   shape, DIRECTION_ROW).
// "hybrid" runs the same product as one spmm_hybrid_csrmm_ex_f32 call (the
// library's own sequencing of the two parts) and prints its time instead.
// One deliberate difference: with transB = 0 and n % bsize != 0 the
// reference's ldb = n is shorter than the nb * bsize rows bsrmm reads, so
// its last block row of B runs into the next column; here y is laid out with
// ldb = n1 in that case (printed), the same matrix with the rows past n
// never met by a nonzero.
#include <iostream>

#include "driver_common.hpp"

int main(int argc, char* argv[]) {
  if (argc < 7) {
    printf("usage: %s <graph> <bsize> <dim> <rocsparse|cusparse|hybrid> <transposeB 0|1> "
           "<density>\n", argv[0]);
    return 1;
  }
  std::string prefix = "tmp/" + std::string(argv[1]);
  std::cout << prefix << std::endl;
  const int bsize = std::stoi(argv[2]);
  const int dim = std::stoi(argv[3]);
  std::string impl(argv[4]);
  const int transposeB = std::stoi(argv[5]);
  const float density = std::stof(argv[6]);
  if (impl != "rocsparse" && impl != "cusparse" && impl != "hybrid") {
    printf("unknown impl %s\n", impl.c_str());
    return 1;
  }
  if (transposeB != 0 && transposeB != 1) {
    printf("transposeB must be 0 or 1\n");
    return 1;
  }
  std::cout << "csr to adj..." << std::endl;
  std::vector<int> rp, ci;
  load_csr_or_die(prefix, rp, ci);
  const int n = (int)rp.size() - 1;
  const int bnum = bsize * bsize;
  const int nb = (n + bsize - 1) / bsize;
  const int n1 = nb * bsize;
  const float alpha = 1.f, beta = 1.f;
  const spmm_operation_t transB =
      transposeB == 0 ? SPMM_OPERATION_NON_TRANSPOSE : SPMM_OPERATION_TRANSPOSE;
  int ldb = transposeB == 0 ? n : dim;
  if (transposeB == 0 && n1 != n) {
    ldb = n1;
    printf("note: ldb = n1 = %d (the reference's ldb = n = %d is short of the %d rows bsrmm "
           "reads)\n", n1, n, n1);
  }

  std::cout << "divide matrix..." << std::endl;
  std::vector<float> ones(ci.size(), 1.f);
  std::vector<int> crp(n + 1), brp(nb + 1);
  int csrNnz = 0, bsrNnzb = 0;
  HANDLE_SPMM_ERROR(spmm_divide_nnz(n, rp.data(), ci.data(), bsize, density, crp.data(),
                                    brp.data(), &csrNnz, &bsrNnzb));
  std::vector<int> cci(csrNnz), bci(bsrNnzb);
  std::vector<float> cval(csrNnz), bval((size_t)bsrNnzb * bnum);
  HANDLE_SPMM_ERROR(spmm_sdivide(n, rp.data(), ci.data(), ones.data(), bsize, density,
                                 crp.data(), brp.data(), cci.data(), cval.data(), bci.data(),
                                 bval.data()));
  printf("csr nnz = %d    bsr nnzb = %d\n", csrNnz, bsrNnzb);

  std::cout << "vec2ptr..." << std::endl;
  std::cout << "gpu memory malloc and memcpy..." << std::endl;
  DeviceArena mem;
  int* d_crp = mem.upload(crp.data(), crp.size());
  int* d_cci = mem.upload(cci.data(), cci.size());
  float* d_cval = mem.upload(cval.data(), cval.size());
  int* d_brp = mem.upload(brp.data(), brp.size());
  int* d_bci = mem.upload(bci.data(), bci.size());
  float* d_bval = mem.upload(bval.data(), bval.size());

  std::cout << "prepare y and z..." << std::endl;
  std::vector<float> y = random_dense(n1, dim);  // n1 * dim values, read with ldb
  float* d_y = mem.upload(y.data(), y.size());
  float* d_z = mem.alloc<float>((size_t)n1 * dim);
  HANDLE_ERROR(hipMemset(d_z, 0, (size_t)n1 * dim * sizeof(float)));

  spmm_handle_t handle = nullptr;
  spmm_mat_descr_t csrDescr = nullptr, bsrDescr = nullptr;
  HANDLE_SPMM_ERROR(spmm_create(&handle));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&csrDescr));
  HANDLE_SPMM_ERROR(spmm_create_mat_descr(&bsrDescr));

  if (impl == "hybrid") {
    EventTimer tm;
    tm.start();
    HANDLE_SPMM_ERROR(spmm_hybrid_csrmm_ex_f32(
        handle, n, dim, n, alpha, d_crp, d_cci, d_cval, csrNnz, bsize, d_brp, d_bci, d_bval,
        bsrNnzb, d_y, ldb, transposeB == 0 ? SPMM_ORDER_COL : SPMM_ORDER_ROW, beta, d_z, n1,
        SPMM_ORDER_COL));
    printf("hybrid cost time:  %3.10f ms \n", tm.stop_ms());
  } else {
    EventTimer t1, t2;
    t1.start();
    HANDLE_SPMM_ERROR(spmm_scsrmm2(handle, SPMM_OPERATION_NON_TRANSPOSE, transB, n, dim, n,
                                   csrNnz, &alpha, csrDescr, d_cval, d_crp, d_cci, d_y, ldb,
                                   &beta, d_z, n1));
    const float time1 = t1.stop_ms();
    t2.start();
    if (impl == "rocsparse") {
      HANDLE_SPMM_ERROR(rocsparse_bsrmm_template<float>(
          handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE, transB, nb, dim, nb, bsrNnzb,
          alpha, bsrDescr, d_bval, d_brp, d_bci, bsize, d_y, ldb, beta, d_z, n1));
    } else {
      HANDLE_SPMM_ERROR(spmm_sbsrmm(handle, SPMM_DIRECTION_ROW, SPMM_OPERATION_NON_TRANSPOSE,
                                    transB, nb, dim, nb, bsrNnzb, &alpha, bsrDescr, d_bval,
                                    d_brp, d_bci, bsize, d_y, ldb, &beta, d_z, n1));
    }
    const float time2 = t2.stop_ms();
    printf("csrmm cost time:  %3.10f ms \n", time1);
    printf("bsrmm cost time:  %3.10f ms \n", time2);
    printf("total cost time:  %3.10f ms \n", time1 + time2);
    printf("%3.5f+%3.5f=%3.5f\n", time1, time2, time1 + time2);
  }
  {  // z is column-major (ldc = n1): rows 0 .. n-1, row-major for the dump
    std::vector<float> zc((size_t)n1 * dim), z((size_t)n * dim);
    HANDLE_ERROR(hipMemcpy(zc.data(), d_z, zc.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < dim; ++c) z[(size_t)r * dim + c] = zc[(size_t)c * n1 + r];
    dump_result(z);
  }
  spmm_destroy_mat_descr(bsrDescr);
  spmm_destroy_mat_descr(csrDescr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
