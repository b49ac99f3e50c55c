// prep.cpp — host-side preprocessing: csr2bsr, bsr2csr, nnzb, row partition.
//
// north_star keeps format conversion as CPU-side preprocessing; these replace
// the GPU cuSPARSE conversions of the reference drivers:
//   cusparseXcsr2bsrNnz + cusparseScsr2bsr   run_bsrmm.cu:116-142, csr2bsr.cu:176-192
//   cusparseSbsr2csr                         bsr2csr.cu:177-188
//   calculateNnzb                            utility.cc:47-69
// and the CPU block extraction of divide_matrix (divide.cu:52-127) at
// density -> 0. Index arrays are bit-exact with the oracle (tests/test_prep.py).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>

#include "host_util.hpp"

#include "spmm_hip.h"

namespace {

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// Collects the sorted distinct block columns of block row `br`.
// `mark` has nb entries, all -1 on entry and on exit.
// Returns false on a column index outside [0, nb*bs).
bool block_cols(int br, int bs, int m, const int* rowptr, const int* colind, int base,
                std::vector<int>& mark, std::vector<int>& out) {
  out.clear();
  const int r0 = br * bs, r1 = std::min(m, r0 + bs);
  const int nb = (int)mark.size();
  for (int r = r0; r < r1; ++r) {
    for (int j = rowptr[r] - base; j < rowptr[r + 1] - base; ++j) {
      const int c = colind[j] - base;
      if (c < 0 || c / bs >= nb) {
        for (int bc : out) mark[bc] = -1;
        return false;
      }
      const int bc = c / bs;
      if (mark[bc] < 0) {
        mark[bc] = 0;
        out.push_back(bc);
      }
    }
  }
  for (int bc : out) mark[bc] = -1;
  std::sort(out.begin(), out.end());
  return true;
}

}  // namespace

extern "C" {

// Block rows are independent: counts and fills run on worker threads (each
// with its own marker array), the prefix sums in between are sequential.
spmm_status_t spmm_xcsr2bsr_nnz(spmm_direction_t dir, int m, int n, const int* csrRowPtr,
                                const int* csrColInd, int blockDim, int* bsrRowPtr,
                                int* nnzbTotal) {
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (m < 0 || n < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!csrRowPtr || !bsrRowPtr || !nnzbTotal) return SPMM_STATUS_INVALID_VALUE;
  const int mb = ceil_div(m, blockDim), nb = ceil_div(n, blockDim);
  if (m > 0 && csrRowPtr[m] - csrRowPtr[0] > 0 && !csrColInd) return SPMM_STATUS_INVALID_VALUE;
  const int base = m > 0 ? csrRowPtr[0] : 0;
  std::vector<int> cnt(mb);
  std::atomic<bool> ok{true};
  spmm_host::parallel_for(mb, [&](int64_t lo, int64_t hi) {
    std::vector<int> mark(std::max(nb, 1), -1), cols;
    for (int64_t br = lo; br < hi && ok; ++br) {
      if (!block_cols((int)br, blockDim, m, csrRowPtr, csrColInd, base, mark, cols)) ok = false;
      cnt[br] = (int)cols.size();
    }
  });
  if (!ok) return SPMM_STATUS_INVALID_VALUE;
  bsrRowPtr[0] = 0;
  long long acc = 0;
  for (int br = 0; br < mb; ++br) {
    acc += cnt[br];
    if (acc > INT32_MAX) return SPMM_STATUS_INVALID_VALUE;
    bsrRowPtr[br + 1] = (int)acc;
  }
  *nnzbTotal = (int)acc;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_scsr2bsr(spmm_direction_t dir, int m, int n, const float* csrVal,
                            const int* csrRowPtr, const int* csrColInd, int blockDim,
                            const int* bsrRowPtr, float* bsrVal, int* bsrColInd) {
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (m < 0 || n < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!csrRowPtr || !bsrRowPtr) return SPMM_STATUS_INVALID_VALUE;
  const int bs = blockDim;
  const int mb = ceil_div(m, bs), nb = ceil_div(n, bs);
  const int nnzb = bsrRowPtr[mb];
  if (nnzb > 0 && (!bsrVal || !bsrColInd || !csrColInd || !csrVal))
    return SPMM_STATUS_INVALID_VALUE;
  const int base = m > 0 ? csrRowPtr[0] : 0;
  const size_t bs2 = (size_t)bs * bs;
  std::atomic<bool> ok{true};
  spmm_host::parallel_for(mb, [&](int64_t lo, int64_t hi) {
    std::vector<int> mark(std::max(nb, 1), -1), cols;
    for (int64_t br = lo; br < hi && ok; ++br) {
      if (!block_cols((int)br, bs, m, csrRowPtr, csrColInd, base, mark, cols)) {
        ok = false;
        return;
      }
      const int k0 = bsrRowPtr[br];
      if (bsrRowPtr[br + 1] - k0 != (int)cols.size()) {
        ok = false;
        return;
      }
      for (size_t t = 0; t < cols.size(); ++t) {
        bsrColInd[k0 + t] = cols[t];
        mark[cols[t]] = k0 + (int)t;
      }
      std::memset(bsrVal + (size_t)k0 * bs2, 0, cols.size() * bs2 * sizeof(float));
      const int r0 = (int)br * bs, r1 = std::min(m, r0 + bs);
      for (int r = r0; r < r1; ++r) {
        const int rr = r - r0;
        for (int j = csrRowPtr[r] - base; j < csrRowPtr[r + 1] - base; ++j) {
          const int c = csrColInd[j] - base;
          const int k = mark[c / bs], cc = c % bs;
          const size_t off = (size_t)k * bs2 + (dir == SPMM_DIRECTION_ROW
                                                    ? (size_t)rr * bs + cc
                                                    : (size_t)cc * bs + rr);
          bsrVal[off] += csrVal[j];  // duplicates summed, in CSR order
        }
      }
      for (int bc : cols) mark[bc] = -1;
    }
  });
  return ok ? SPMM_STATUS_SUCCESS : SPMM_STATUS_INVALID_VALUE;
}

spmm_status_t spmm_sbsr2csr(spmm_direction_t dir, int mb, int nb, const float* bsrVal,
                            const int* bsrRowPtr, const int* bsrColInd, int blockDim,
                            float* csrVal, int* csrRowPtr, int* csrColInd) {
  if (dir != SPMM_DIRECTION_ROW && dir != SPMM_DIRECTION_COLUMN) return SPMM_STATUS_INVALID_VALUE;
  if (mb < 0 || nb < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!bsrRowPtr || !csrRowPtr) return SPMM_STATUS_INVALID_VALUE;
  const int bs = blockDim;
  const size_t bs2 = (size_t)bs * bs;
  const int base = mb > 0 ? bsrRowPtr[0] : 0;
  if (mb > 0 && bsrRowPtr[mb] - base > 0 && (!bsrVal || !bsrColInd || !csrVal || !csrColInd))
    return SPMM_STATUS_INVALID_VALUE;
  long long pos = 0;
  csrRowPtr[0] = 0;
  for (int br = 0; br < mb; ++br) {
    const int k0 = bsrRowPtr[br] - base, k1 = bsrRowPtr[br + 1] - base;
    for (int rr = 0; rr < bs; ++rr) {
      for (int k = k0; k < k1; ++k) {
        const long long cb = (long long)(bsrColInd[k] - base) * bs;
        const float* blk = bsrVal + (size_t)k * bs2;
        for (int c = 0; c < bs; ++c) {
          csrColInd[pos] = (int)(cb + c);
          csrVal[pos] = dir == SPMM_DIRECTION_ROW ? blk[(size_t)rr * bs + c]
                                                  : blk[(size_t)c * bs + rr];
          ++pos;
        }
      }
      if (pos > INT32_MAX) return SPMM_STATUS_INVALID_VALUE;
      csrRowPtr[(size_t)br * bs + rr + 1] = (int)pos;
    }
  }
  (void)nb;
  return SPMM_STATUS_SUCCESS;
}

int64_t spmm_calculate_nnzb(int n, const int* csrRowPtr, const int* csrColInd, int blockDim) {
  if (n < 0 || blockDim <= 0 || !csrRowPtr) return -1;
  const int mb = ceil_div(n, blockDim);
  const int base = n > 0 ? csrRowPtr[0] : 0;
  int maxc = 0;
  for (int j = 0; j < csrRowPtr[n] - base; ++j) maxc = std::max(maxc, csrColInd[j] - base);
  const int nb = std::max(ceil_div(n, blockDim), maxc / blockDim + 1);
  std::vector<int> mark(std::max(nb, 1), -1), cols;
  int64_t total = 0;
  for (int br = 0; br < mb; ++br) {
    if (!block_cols(br, blockDim, n, csrRowPtr, csrColInd, base, mark, cols)) return -1;
    total += (int64_t)cols.size();
  }
  return total;
}

spmm_status_t spmm_csr_partition_rows(int m, const int* csrRowPtr, int nparts, int* bounds) {
  if (m < 0 || nparts <= 0 || !csrRowPtr || !bounds) return SPMM_STATUS_INVALID_VALUE;
  // Cost of the prefix [0, i) = nnz before row i + i (one unit per row for
  // its output write), monotone in i: cut at equal cost quantiles.
  const long long base = csrRowPtr[0];
  const long long total = (long long)csrRowPtr[m] - base + m;
  bounds[0] = 0;
  for (int p = 1; p < nparts; ++p) {
    const long long target = (total * p) / nparts;
    int lo = bounds[p - 1], hi = m;
    while (lo < hi) {  // first i with cost(i) >= target
      const int mid = lo + (hi - lo) / 2;
      const long long cost = (long long)csrRowPtr[mid] - base + mid;
      if (cost < target) lo = mid + 1; else hi = mid;
    }
    bounds[p] = lo;
  }
  bounds[nparts] = m;
  return SPMM_STATUS_SUCCESS;
}

}  // extern "C"

// ----------------------------------------------------------------------------
// divide_matrix (divide.cu:52-127) with values.
// ----------------------------------------------------------------------------
namespace {

// Per block row: entry counts per block column (over the block row's rows),
// and the admitted block columns in ascending order. `cnt` has nb entries,
// zero on entry and on exit; `touched` lists the columns with a count.
struct DivideScratch {
  std::vector<int> cnt, touched, slot;
  explicit DivideScratch(int nb) : cnt(std::max(nb, 1), 0), slot(std::max(nb, 1), -1) {}
};

// Returns false on an out-of-range column. Fills `adm` with the admitted
// block columns (ascending).
bool divide_block_row(int br, int bs, int n, int nb, const int* rowptr, const int* colind,
                      int base, float density, DivideScratch& s, std::vector<int>& adm) {
  adm.clear();
  s.touched.clear();
  const int r0 = br * bs, r1 = std::min(n, r0 + bs);
  for (int r = r0; r < r1; ++r)
    for (int j = rowptr[r] - base; j < rowptr[r + 1] - base; ++j) {
      const int c = colind[j] - base;
      if (c < 0 || c / bs >= nb) {
        for (int t : s.touched) s.cnt[t] = 0;
        return false;
      }
      if (s.cnt[c / bs]++ == 0) s.touched.push_back(c / bs);
    }
  const double bnum = (double)bs * bs;
  if (density <= 0.f) {
    // 0 >= 0: every block column is admitted, empty ones included (divide.cu:91).
    for (int bc = 0; bc < nb; ++bc) adm.push_back(bc);
  } else {
    for (int bc : s.touched)
      if ((float)(s.cnt[bc] / bnum) >= density) adm.push_back(bc);
    std::sort(adm.begin(), adm.end());
  }
  for (int t : s.touched) s.cnt[t] = 0;
  return true;
}

}  // namespace

extern "C" {

spmm_status_t spmm_divide_nnz(int n, const int* rowPtr, const int* colInd, int blockDim,
                              float density, int* csrRowPtr, int* bsrRowPtr, int* csrNnz,
                              int* nnzb) {
  if (n < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!rowPtr || !csrRowPtr || !bsrRowPtr || !csrNnz || !nnzb) return SPMM_STATUS_INVALID_VALUE;
  const int bs = blockDim, nb = ceil_div(n, bs), mb = nb;
  const int base = n > 0 ? rowPtr[0] : 0;
  if (n > 0 && rowPtr[n] - base > 0 && !colInd) return SPMM_STATUS_INVALID_VALUE;
  // Per block row (worker threads): admitted blocks, and per CSR row the
  // entries left to the remainder (stored in csrRowPtr[r + 1], summed below).
  std::vector<int> nb_row(mb);
  std::atomic<bool> ok{true};
  spmm_host::parallel_for(mb, [&](int64_t lo, int64_t hi) {
    DivideScratch s(nb);
    std::vector<int> adm;
    for (int64_t br = lo; br < hi && ok; ++br) {
      if (!divide_block_row((int)br, bs, n, nb, rowPtr, colInd, base, density, s, adm)) {
        ok = false;
        return;
      }
      nb_row[br] = (int)adm.size();
      for (int bc : adm) s.slot[bc] = 1;
      const int r0 = (int)br * bs, r1 = std::min(n, r0 + bs);
      for (int r = r0; r < r1; ++r) {
        int c = 0;
        for (int j = rowPtr[r] - base; j < rowPtr[r + 1] - base; ++j)
          if (s.slot[(colInd[j] - base) / bs] < 0) ++c;
        csrRowPtr[r + 1] = c;
      }
      for (int bc : adm) s.slot[bc] = -1;
    }
  });
  if (!ok) return SPMM_STATUS_INVALID_VALUE;
  long long nb_acc = 0, c_acc = 0;
  csrRowPtr[0] = 0;
  bsrRowPtr[0] = 0;
  for (int r = 0; r < n; ++r) {
    c_acc += csrRowPtr[r + 1];
    if (c_acc > INT32_MAX) return SPMM_STATUS_INVALID_VALUE;
    csrRowPtr[r + 1] = (int)c_acc;
  }
  for (int br = 0; br < mb; ++br) {
    nb_acc += nb_row[br];
    if (nb_acc > INT32_MAX) return SPMM_STATUS_INVALID_VALUE;
    bsrRowPtr[br + 1] = (int)nb_acc;
  }
  *csrNnz = (int)c_acc;
  *nnzb = (int)nb_acc;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_sdivide(int n, const int* rowPtr, const int* colInd, const float* val,
                           int blockDim, float density, const int* csrRowPtr,
                           const int* bsrRowPtr, int* csrColInd, float* csrVal, int* bsrColInd,
                           float* bsrVal) {
  if (n < 0 || blockDim <= 0) return SPMM_STATUS_INVALID_VALUE;
  if (!rowPtr || !csrRowPtr || !bsrRowPtr) return SPMM_STATUS_INVALID_VALUE;
  const int bs = blockDim, nb = ceil_div(n, bs), mb = nb;
  const int base = n > 0 ? rowPtr[0] : 0;
  if (n > 0 && rowPtr[n] - base > 0 && (!colInd || !val)) return SPMM_STATUS_INVALID_VALUE;
  if ((csrRowPtr[n] > 0 && (!csrColInd || !csrVal)) ||
      (bsrRowPtr[mb] > 0 && (!bsrColInd || !bsrVal)))
    return SPMM_STATUS_INVALID_VALUE;
  const size_t bs2 = (size_t)bs * bs;
  std::atomic<bool> ok{true};
  spmm_host::parallel_for(mb, [&](int64_t lo, int64_t hi) {
    DivideScratch s(nb);
    std::vector<int> adm;
    for (int64_t br = lo; br < hi && ok; ++br) {
      if (!divide_block_row((int)br, bs, n, nb, rowPtr, colInd, base, density, s, adm)) {
        ok = false;
        return;
      }
      const int k0 = bsrRowPtr[br];
      if (bsrRowPtr[br + 1] - k0 != (int)adm.size()) {
        ok = false;
        return;
      }
      for (size_t t = 0; t < adm.size(); ++t) {
        bsrColInd[k0 + t] = adm[t];
        s.slot[adm[t]] = k0 + (int)t;
      }
      if (!adm.empty())
        std::memset(bsrVal + (size_t)k0 * bs2, 0, adm.size() * bs2 * sizeof(float));
      const int r0 = (int)br * bs, r1 = std::min(n, r0 + bs);
      for (int r = r0; r < r1; ++r) {
        int pos = csrRowPtr[r];
        for (int j = rowPtr[r] - base; j < rowPtr[r + 1] - base; ++j) {
          const int c = colInd[j] - base;
          const int k = s.slot[c / bs];
          if (k < 0) {
            csrColInd[pos] = c;
            csrVal[pos] = val[j];
            ++pos;
          } else {
            bsrVal[(size_t)k * bs2 + (size_t)(r - r0) * bs + c % bs] += val[j];
          }
        }
        if (pos != csrRowPtr[r + 1]) ok = false;
      }
      for (int bc : adm) s.slot[bc] = -1;
    }
  });
  return ok ? SPMM_STATUS_SUCCESS : SPMM_STATUS_INVALID_VALUE;
}

spmm_status_t spmm_hybrid_plan(int n, const int* rowPtr, const int* colInd, int blockDim, int K,
                               int valueBytes, double bsrBytesPerSec, double csrBytesPerSec,
                               float* density, int64_t* nnzb, int64_t* csrNnz,
                               double* estSeconds) {
  if (n < 0 || blockDim <= 0 || K <= 0 || valueBytes <= 0 || !rowPtr || !density)
    return SPMM_STATUS_INVALID_VALUE;
  const int bs = blockDim, nb = ceil_div(n, bs);
  const int64_t bs2 = (int64_t)bs * bs;
  const int base = n > 0 ? rowPtr[0] : 0;
  if (n > 0 && rowPtr[n] - base > 0 && !colInd) return SPMM_STATUS_INVALID_VALUE;
  const double bw_b = bsrBytesPerSec > 0 ? bsrBytesPerSec : 7.0e12;
  const double bw_c = csrBytesPerSec > 0 ? csrBytesPerSec : 7.5e12;
  // hist[c] = number of blocks holding c entries (c = 1 .. bs^2; duplicates
  // counted, as divide_matrix counts them).
  const int nt = spmm_host::num_threads();
  std::vector<std::vector<int64_t>> hist(nt, std::vector<int64_t>(bs2 + 1, 0));
  std::atomic<bool> ok{true};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      DivideScratch s(nb);
      auto& h = hist[t];
      for (int br = (int)((int64_t)nb * t / nt); br < (int)((int64_t)nb * (t + 1) / nt); ++br) {
        s.touched.clear();
        const int r0 = br * bs, r1 = std::min(n, r0 + bs);
        for (int r = r0; r < r1; ++r)
          for (int j = rowPtr[r] - base; j < rowPtr[r + 1] - base; ++j) {
            const int c = colInd[j] - base;
            if (c < 0 || c / bs >= nb) {
              ok = false;
              for (int x : s.touched) s.cnt[x] = 0;
              return;
            }
            if (s.cnt[c / bs]++ == 0) s.touched.push_back(c / bs);
          }
        for (int x : s.touched) {
          ++h[std::min<int64_t>(s.cnt[x], bs2)];
          s.cnt[x] = 0;
        }
      }
    });
  for (auto& x : th) x.join();
  if (!ok) return SPMM_STATUS_INVALID_VALUE;
  for (int t = 1; t < nt; ++t)
    for (int64_t c = 0; c <= bs2; ++c) hist[0][c] += hist[t][c];
  const auto& h = hist[0];
  const double tb = ((double)valueBytes * (bs2 + (double)bs * K) + 4.0) / bw_b;
  const double tn = (8.0 + 4.0 * K) / bw_c;
  // T = bs^2 + 1 (all CSR) first; lowering T moves the blocks of fill T - 1
  // from the CSR side to the BSR side.
  int64_t total_nnz = 0;
  for (int64_t c = 1; c <= bs2; ++c) total_nnz += c * h[c];
  double cost = total_nnz * tn, best = cost;
  int64_t bestT = bs2 + 1, blocks = 0, rem = total_nnz, best_blocks = 0, best_rem = rem;
  for (int64_t T = bs2; T >= 1; --T) {
    cost += h[T] * (tb - T * tn);
    blocks += h[T];
    rem -= T * h[T];
    if (cost < best) {
      best = cost;
      bestT = T;
      best_blocks = blocks;
      best_rem = rem;
    }
  }
  *density = (float)((double)bestT / (double)bs2);
  if (nnzb) *nnzb = best_blocks;
  if (csrNnz) *csrNnz = best_rem;
  if (estSeconds) *estSeconds = best;
  return SPMM_STATUS_SUCCESS;
}

}  // extern "C"

