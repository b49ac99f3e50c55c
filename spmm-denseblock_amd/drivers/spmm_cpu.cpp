// spmm_cpu [N] [p] [K] [reps]   — the reference's CPU path (spmm.cc) as a driver.
//
// spmm.cc does not build as shipped (it includes a matrix.h that is not in
// the tree, spmm.cc:5); this restates its csr_spmm (spmm.cc:7-25): OpenMP
// over rows, output column k OUTER and the row's nnz INNER, pattern only
// (unit values), double dense/out, row-major. BASELINE configs[0]: N = 16384,
// p = 2^-10 (randomCSRMatrix from the shared mt19937_64, ~256K nnz), K = 32.
// Also runs spmm.cc's small tests (spmm.cc:45-61; expected [[4,6,7],[8,17,3]])
// and times coo_spmm (spmm.cc:27-43) on the same matrix, as spmm.cc's main does.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "spmm_host.h"

// spmm.cc:27-43 coo_spmm: out zeroed, OpenMP over the nnz entries, `omp atomic`
// adds of the dense row into the output row.
static void coo_spmm(int64_t rows, int64_t nnz, const int64_t* row, const int64_t* col,
                     const double* dense, int64_t dcols, double* out) {
  std::fill(out, out + rows * dcols, 0.0);
#pragma omp parallel for
  for (int64_t i = 0; i < nnz; ++i) {
    double* o = out + row[i] * dcols;
    const double* d = dense + col[i] * dcols;
    for (int64_t k = 0; k < dcols; ++k) {
#pragma omp atomic
      o[k] += d[k];
    }
  }
}

static void csr_spmm(int64_t rows, const int64_t* indptr, const int64_t* indices,
                     const double* dense, int64_t dcols, double* out) {
#pragma omp parallel for
  for (int64_t rid = 0; rid < rows; ++rid) {
    const int64_t s = indptr[rid], e = indptr[rid + 1];
    double* o = out + rid * dcols;
    for (int64_t k = 0; k < dcols; ++k) {
      double acc = 0;
      for (int64_t j = s; j < e; ++j) acc += dense[indices[j] * dcols + k];
      o[k] = acc;
    }
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::stoi(argv[1]) : 16384;
  const float p = argc > 2 ? std::stof(argv[2]) : 1.0f / 1024;
  const int K = argc > 3 ? std::stoi(argv[3]) : 32;
  const int reps = argc > 4 ? std::stoi(argv[4]) : 5;
  {  // spmm.cc:45-52
    const int64_t ip[] = {0, 1, 3}, ix[] = {1, 0, 2};
    const double d[] = {3, 9, 2, 4, 6, 7, 5, 8, 1};
    double o[6];
    csr_spmm(2, ip, ix, d, 3, o);
    printf("small csr_spmm: [[%g,%g,%g],[%g,%g,%g]]\n", o[0], o[1], o[2], o[3], o[4], o[5]);
    const int64_t cr[] = {0, 1, 1};  // spmm.cc:56
    coo_spmm(2, 3, cr, ix, d, 3, o);
    printf("small coo_spmm: [[%g,%g,%g],[%g,%g,%g]]\n", o[0], o[1], o[2], o[3], o[4], o[5]);
  }
  std::vector<int> rp(N + 1);
  int* ci = nullptr;
  float* v = nullptr;
  const int64_t nnz = spmm_host_random_csr(N, N, p, -1.f, 1.f, rp.data(), &ci, &v);
  std::vector<int64_t> ip(rp.begin(), rp.end()), ix(ci, ci + nnz);
  spmm_host_free(ci);
  spmm_host_free(v);
  std::vector<float> df((size_t)N * K);
  spmm_host_random_array((int64_t)N * K, -1.f, 1.f, df.data());
  std::vector<double> dense(df.begin(), df.end()), out((size_t)N * K);
  csr_spmm(N, ip.data(), ix.data(), dense.data(), K, out.data());  // warm-up
  std::vector<double> ts;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::high_resolution_clock::now();
    csr_spmm(N, ip.data(), ix.data(), dense.data(), K, out.data());
    auto t1 = std::chrono::high_resolution_clock::now();
    ts.push_back(std::chrono::duration<double>(t1 - t0).count());
  }
  std::sort(ts.begin(), ts.end());
  const double med = ts[ts.size() / 2];
  printf("N=%d nnz=%lld K=%d threads=%d\n", N, (long long)nnz, K, omp_get_max_threads());
  printf("csr_spmm time cost: %gs\n", med);
  printf("GFLOP/s (2*nnz*K/t): %.3f\n", 2.0 * nnz * K / med / 1e9);
  {  // spmm.cc:27-43 / :75-85: the same product from COO
    std::vector<int64_t> row(nnz);
    for (int r = 0; r < N; ++r)
      for (int64_t j = ip[r]; j < ip[r + 1]; ++j) row[j] = r;
    std::vector<double> out2((size_t)N * K);
    coo_spmm(N, nnz, row.data(), ix.data(), dense.data(), K, out2.data());  // warm-up
    std::vector<double> tc;
    for (int r = 0; r < reps; ++r) {
      auto t0 = std::chrono::high_resolution_clock::now();
      coo_spmm(N, nnz, row.data(), ix.data(), dense.data(), K, out2.data());
      auto t1 = std::chrono::high_resolution_clock::now();
      tc.push_back(std::chrono::duration<double>(t1 - t0).count());
    }
    std::sort(tc.begin(), tc.end());
    double maxdiff = 0;
    for (size_t i = 0; i < out.size(); ++i) maxdiff = std::max(maxdiff, std::fabs(out[i] - out2[i]));
    printf("coo_spmm time cost: %gs\n", tc[tc.size() / 2]);
    printf("coo GFLOP/s (2*nnz*K/t): %.3f  max |csr - coo| = %.3g\n",
           2.0 * nnz * K / tc[tc.size() / 2] / 1e9, maxdiff);
  }
  return 0;
}
