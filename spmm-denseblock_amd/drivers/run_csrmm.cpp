// run_csrmm <graph> <dim> <impl> <transposeB> [--gpus N] [--chunks C]
// Reference CLI of run_csrmm.cu:46-171 on the HIP engine. Reads
// tmp/<graph>_indptr.txt / _indices.txt, values 1.0, B = randomDenseMatrix
// (mt19937_64 seeded 1234), times 10 epochs with events on stream 0 and
// prints the reference's lines. impl: gespmm (gespmm_csrmm<float>), gespmm_hot
// (the same layout on hot-column hints, tagged once before the epochs),
// cusparseScsrmm (col-major B and C), cusparseScsrmm2 (transposeB picks the
// B layout, col-major C) — all served by libspmm_hip.so.
// --gpus N (impl gespmm; not in the reference, which is single-GPU): the rows
// are cut into N nnz-balanced shards (spmm_csr_partition_rows), one per GPU
// of this process, B replicated, and C assembled on every GPU by the RCCL
// exchange of spmm_csr_f32_multi (include/spmm_multi.h: grouped send / recv
// of exact row shards into each GPU's n x dim C), C chunks overlapping the
// next chunk's compute. Every mode ends with a checksum of C.
#include <cassert>
#include <chrono>
#include <iostream>

#include "driver_common.hpp"
#include "spmm_multi.h"

static void print_checksum(const std::vector<float>& z, int n, int dim) {
  double sum = 0.0, asum = 0.0;
  for (float x : z) {
    sum += x;
    asum += x < 0 ? -x : x;
  }
  printf("C checksum: sum=%.9e abssum=%.9e C[0][0..1]=%.9g %.9g C[n-1][dim-1]=%.9g\n", sum, asum,
         z[0], dim > 1 ? z[1] : 0.f, z[(size_t)n * dim - 1]);
}

// N GPUs of this process: shards, replicas, the multi-GPU call, timing.
static int run_multi(int ngpu, int chunks, const std::vector<int>& rp, const std::vector<int>& ci,
                     const std::vector<float>& val, const std::vector<float>& y, int dim) {
  const int n = (int)rp.size() - 1;
  std::vector<int> bounds(ngpu + 1);
  HANDLE_SPMM_ERROR(spmm_csr_partition_rows(n, rp.data(), ngpu, bounds.data()));
  const int slot = spmm_multi_slot_rows(ngpu, bounds.data(), chunks);
  printf("multi-GPU: ngpu=%d chunks=%d chunk_rows=%d rows/part:", ngpu, chunks, slot);
  for (int p = 0; p < ngpu; ++p) printf(" %d", bounds[p + 1] - bounds[p]);
  printf("\n");
  DeviceArena mem;
  std::vector<const int*> drp(ngpu), dci(ngpu);
  std::vector<const float*> dv(ngpu), dB(ngpu);
  std::vector<float*> dC(ngpu);
  std::vector<int> part_nnz(ngpu);
  const size_t cfloats = (size_t)n * dim;
  for (int p = 0; p < ngpu; ++p) {
    HANDLE_ERROR(hipSetDevice(p));
    const int r0 = bounds[p], r1 = bounds[p + 1], j0 = rp[r0], j1 = rp[r1];
    std::vector<int> lrp(rp.begin() + r0, rp.begin() + r1 + 1);
    for (int& x : lrp) x -= j0;
    part_nnz[p] = j1 - j0;
    drp[p] = mem.upload(lrp.data(), lrp.size());
    dci[p] = mem.upload(ci.data() + j0, (size_t)(j1 - j0));
    dv[p] = mem.upload(val.data() + j0, (size_t)(j1 - j0));
    dB[p] = mem.upload(y.data(), y.size());
    dC[p] = mem.alloc<float>(cfloats);
    HANDLE_ERROR(hipMemset(dC[p], 0, cfloats * sizeof(float)));
  }
  HANDLE_ERROR(hipSetDevice(0));
  spmm_multi_t ctx = nullptr;
  HANDLE_SPMM_ERROR(spmm_multi_create(&ctx, ngpu, nullptr));
  HANDLE_SPMM_ERROR(spmm_multi_set_timing(ctx, 1));
  printf("csrmm...\n");
  const int epoch = 10;
  float total = 0.f, comp_max = 0.f, tot_max = 0.f;
  std::vector<float> comp(ngpu), tot(ngpu);
  for (int i = 0; i < epoch; ++i) {
    auto t0 = std::chrono::high_resolution_clock::now();
    HANDLE_SPMM_ERROR(spmm_csr_f32_multi(ctx, n, dim, n, bounds.data(), drp.data(), dci.data(),
                                         dv.data(), part_nnz.data(), dB.data(), dim, dC.data(),
                                         dim, chunks));
    HANDLE_SPMM_ERROR(spmm_multi_synchronize(ctx));
    auto t1 = std::chrono::high_resolution_clock::now();
    const float t = std::chrono::duration<float, std::milli>(t1 - t0).count();
    HANDLE_SPMM_ERROR(spmm_multi_get_times(ctx, comp.data(), tot.data()));
    float cm = 0.f, tm = 0.f;
    for (int p = 0; p < ngpu; ++p) {
      cm = std::max(cm, comp[p]);
      tm = std::max(tm, tot[p]);
    }
    printf("csrmm cost time:  %3.10f ms  (max over GPUs: compute %.4f ms, compute + exchange "
           "%.4f ms)\n", t, cm, tm);
    total += t;
    comp_max += cm;
    tot_max += tm;
  }
  const float avg = total / epoch;
  printf("average csrmm cost time: %3.10f ms\n", avg);
  printf("average per-GPU compute %.4f ms, compute + exchange %.4f ms\n", comp_max / epoch,
         tot_max / epoch);
  printf("GFLOP/s (2*nnz*dim/t): %6.3f\n", 2.0 * (double)rp[n] * dim / (avg * 1e6));
  // C on the last GPU (every GPU holds all of it, row-major n x dim)
  std::vector<float> z(cfloats);
  HANDLE_ERROR(hipSetDevice(ngpu - 1));
  HANDLE_ERROR(hipMemcpy(z.data(), dC[ngpu - 1], cfloats * sizeof(float), hipMemcpyDeviceToHost));
  print_checksum(z, n, dim);
  dump_result(z);
  spmm_multi_destroy(ctx);
  printf("end\n");
  return 0;
}

int main(int argc, char* argv[]) {
  int ngpu = 0, chunks = 1;
  std::vector<char*> pos;
  for (int i = 0; i < argc; ++i) {
    const std::string a(argv[i]);
    if (a == "--gpus" && i + 1 < argc) ngpu = std::stoi(argv[++i]);
    else if (a == "--chunks" && i + 1 < argc) chunks = std::stoi(argv[++i]);
    else pos.push_back(argv[i]);
  }
  argc = (int)pos.size();
  argv = pos.data();
  if (argc < 5) {
    printf("usage: %s <graph> <dim> <gespmm|gespmm_hot|cusparseScsrmm|cusparseScsrmm2> <transposeB> "
           "[--gpus N] [--chunks C]\n",
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
  if (ngpu > 0) {
    if (impl != "gespmm") {
      printf("--gpus runs the gespmm layout (row-major B and C) only\n");
      return 1;
    }
    int ndev = 0;
    HANDLE_ERROR(hipGetDeviceCount(&ndev));
    if (ngpu > ndev || chunks < 1) {
      printf("--gpus %d --chunks %d: %d devices visible\n", ngpu, chunks, ndev);
      return 1;
    }
    return run_multi(ngpu, chunks, rp, ci, val, y, dim);
  }

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
  if (impl != "gespmm" && impl != "gespmm_hot" && transposeB == 0) {
    std::vector<float> yc((size_t)n * dim);
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < dim; ++c) yc[(size_t)c * n + r] = y[(size_t)r * dim + c];
    d_yc = mem.upload(yc.data(), yc.size());
  }
  // gespmm_hot (not in the reference): gespmm's layout on hot-column cache hints,
  // the columns tagged once before the epochs (spmm_csr_hot_analysis)
  int* d_ci_hot = nullptr;
  if (impl == "gespmm_hot") {
    d_ci_hot = mem.alloc<int>(ci.size());
    EventTimer ta;
    ta.start();
    HANDLE_SPMM_ERROR(spmm_csr_hot_analysis(handle, dim, n, nnz, d_ci, SPMM_INDEX_BASE_ZERO, 0,
                                            d_ci_hot));
    printf("hot-column analysis time: %3.10f ms\n", ta.stop_ms());
  }
  printf("csrmm...\n");
  const int epoch = 10;
  float total = 0.f;
  EventTimer tm;
  for (int i = 0; i < epoch; ++i) {
    tm.start();
    if (impl == "gespmm") {
      gespmm_csrmm<float>(n, dim, d_rp, d_ci, d_val, d_y, d_z);
    } else if (impl == "gespmm_hot") {
      HANDLE_SPMM_ERROR(spmm_csrmm_hot_f32(handle, n, dim, n, nnz, 1.f, d_rp, d_ci_hot, d_val,
                                           SPMM_INDEX_BASE_ZERO, d_y, dim, SPMM_ORDER_ROW, 0.f,
                                           d_z, dim, SPMM_ORDER_ROW));
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
  {  // C back to the host, row-major (the cusparse forms write it col-major)
    std::vector<float> zc((size_t)n * dim), z((size_t)n * dim);
    HANDLE_ERROR(hipMemcpy(zc.data(), d_z, zc.size() * sizeof(float), hipMemcpyDeviceToHost));
    if (impl == "gespmm" || impl == "gespmm_hot") z = zc;
    else
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < dim; ++c) z[(size_t)r * dim + c] = zc[(size_t)c * n + r];
    print_checksum(z, n, dim);
    dump_result(z);
  }
  spmm_destroy_mat_descr(descr);
  spmm_destroy(handle);
  printf("end\n");
  return 0;
}
