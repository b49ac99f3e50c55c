// oracle.cpp — CPU restatement of the reference's hot-path semantics.
//
// TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
// (or the timed CPU baseline) — never as part of the product path. The
// product (libspmm_hip.so) never links or calls anything here.
//
// Pinning: the reference's SpMM kernels are CUDA / closed
// cuSPARSE and cannot run here, so absolute SpMM values are pinned by the
// reference's own known-answer programs (csrmm.cu, bsrmm.cu, block_cublas.cu,
// try_cublas.cu, spmm.cc small tests; expected outputs committed under
// tests/golden/) and by documented cuSPARSE semantics. The RNG and the
// csr2bsr/nnzb index arrays are additionally pinned bit-exactly against the
// reference's own host code compiled from /root/reference into oracle/_ref
// (oracle/ref/Makefile) — see tests/test_oracle.py.
//
// Every function names the reference file:line whose semantics it restates.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// Dense element accessors. order 0 = row-major, 1 = column-major.
inline size_t at(int r, int c, int ld, int order) {
  return order == 0 ? (size_t)r * ld + c : (size_t)c * ld + r;
}

std::mt19937_64 g_gen(1234);  // load_data.cc:12 (one generator per process)

}  // namespace

extern "C" {

// ---------------------------------------------------------------- RNG ----
// load_data.cc:12, 29-36: std::mt19937_64 seeded 1234 shared by all calls,
// std::uniform_real_distribution<float>(minVal, maxVal).
void oracle_rng_seed(uint64_t s) { g_gen.seed(s); }

void oracle_random_array(int64_t n, float lo, float hi, float* out) {
  std::uniform_real_distribution<float> dist(lo, hi);
  for (int64_t i = 0; i < n; ++i) out[i] = dist(g_gen);
}

// load_data.cc:42-69 randomCSRMatrix: for each row, for each column, one
// flip(0,1) draw; on a hit (< p) the value is drawn immediately after.
// Writes rowptr[m+1]; colind/val must hold `cap` entries. Returns nnz, or -1
// if cap is too small.
int64_t oracle_random_csr(int m, int n, float p, float lo, float hi, int* rowptr, int* colind,
                          float* val, int64_t cap) {
  std::uniform_real_distribution<float> flip(0, 1), dist(lo, hi);
  int64_t cnt = 0;
  rowptr[0] = 0;
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j < n; ++j) {
      if (flip(g_gen) < p) {
        const float v = dist(g_gen);
        if (cnt >= cap) return -1;
        colind[cnt] = j;
        val[cnt] = v;
        ++cnt;
      }
    }
    rowptr[i + 1] = (int)cnt;
  }
  return cnt;
}

// -------------------------------------------------------------- CSR -----
// Semantics of gespmm_csrmm (gespmm_csrmm.h:116-134: per output element a
// sequential `acc += val * B[col*K + c]` over the row's nnz in CSR order,
// contracted to FMA by nvcc) generalised with cusparseScsrmm's alpha/beta and
// storage orders (run_csrmm.cu:135-142), epilogue as rocsparse_bsrmm_impl.h:
// 381-388 (beta == 0 -> alpha*sum without reading C, else fma(beta, C, alpha*sum)).
// T = double is gespmm_csrmm<double> (the template's T, gespmm_csrmm.h:422).
extern "C++" {
template <class T>
static void csrmm_seq(int m, int n, const int* rowptr, const int* colind, const T* val, int base,
                      const T* B, int ldb, int orderB, T alpha, T beta, T* C, int ldc,
                      int orderC) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int r = 0; r < m; ++r) {
    const int j0 = rowptr[r] - base, j1 = rowptr[r + 1] - base;
    for (int c = 0; c < n; ++c) {
      T acc = 0;
      for (int j = j0; j < j1; ++j)
        acc = std::fma(val[j], B[at(colind[j] - base, c, ldb, orderB)], acc);
      T& out = C[at(r, c, ldc, orderC)];
      out = beta == T(0) ? alpha * acc : std::fma(beta, out, alpha * acc);
    }
  }
}
}  // extern "C++"

void oracle_csrmm_f32(int m, int n, const int* rowptr, const int* colind, const float* val,
                      int base, const float* B, int ldb, int orderB, float alpha, float beta,
                      float* C, int ldc, int orderC) {
  csrmm_seq<float>(m, n, rowptr, colind, val, base, B, ldb, orderB, alpha, beta, C, ldc, orderC);
}

// The association the HIP CSR kernels use, restated so that
// their output can be checked bit for bit at any grid: a row of L nonzeros is
// summed as pieces of T(L) = max(128, ceil(L / 64)) consecutive nonzeros from
// the row's start, each the sequential fp32 FMA chain of csrmm_seq above
// (gespmm_csrmm.h:124-129), and the pieces are added left to right from -0.
// Rows of at most 128 nonzeros are therefore exactly csrmm_seq's chain.
int oracle_csr_piece_len(int L) { return std::max(128, (int)(((unsigned)L + 63u) >> 6)); }

void oracle_csrmm_pieces_f32(int m, int n, const int* rowptr, const int* colind,
                             const float* val, int base, const float* B, int ldb, int orderB,
                             float alpha, float beta, float* C, int ldc, int orderC) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int r = 0; r < m; ++r) {
    const int j0 = rowptr[r] - base, j1 = rowptr[r + 1] - base;
    const int T = oracle_csr_piece_len(j1 - j0);
    for (int c = 0; c < n; ++c) {
      // no reassociation of the piece sums; an empty row is one empty piece, +0 (the
      // reference's accumulator before its first FMA: the kernels' -0 + (+0))
      volatile float x = j1 > j0 ? -0.f : 0.f;
      for (int p = j0; p < j1; p += T) {
        float acc = 0.f;
        for (int j = p; j < std::min(p + T, j1); ++j)
          acc = std::fma(val[j], B[at(colind[j] - base, c, ldb, orderB)], acc);
        x = x + acc;
      }
      float& out = C[at(r, c, ldc, orderC)];
      out = beta == 0.f ? alpha * x : std::fma(beta, out, alpha * x);
    }
  }
}

void oracle_csrmm_d(int m, int n, const int* rowptr, const int* colind, const double* val,
                    int base, const double* B, int ldb, int orderB, double alpha, double beta,
                    double* C, int ldc, int orderC) {
  csrmm_seq<double>(m, n, rowptr, colind, val, base, B, ldb, orderB, alpha, beta, C, ldc, orderC);
}

// Same product in double, plus the per-element magnitude sum |a|.|b| used by
// the norm-wise tolerance |C - C64| <= tol * absdot.
void oracle_csrmm_f64(int m, int n, const int* rowptr, const int* colind, const float* val,
                      int base, const float* B, int ldb, int orderB, double* C, double* absdot) {
  // Nonzeros outer, output columns inner: each output still sums its terms in nonzero
  // order (the same double additions as a column-outer loop, bit for bit), but a row-major
  // B row is read contiguously, so a whole products-sized product checks in seconds.
#pragma omp parallel for schedule(dynamic, 64)
  for (int r = 0; r < m; ++r) {
    const int j0 = rowptr[r] - base, j1 = rowptr[r + 1] - base;
    double* acc = C + (size_t)r * n;
    double* aa = absdot ? absdot + (size_t)r * n : nullptr;
    for (int c = 0; c < n; ++c) {
      acc[c] = 0.0;
      if (aa) aa[c] = 0.0;
    }
    for (int j = j0; j < j1; ++j) {
      const double v = (double)val[j];
      const int row = colind[j] - base;
      for (int c = 0; c < n; ++c) {
        const double t = v * (double)B[at(row, c, ldb, orderB)];
        acc[c] += t;
        if (aa) aa[c] += std::fabs(t);
      }
    }
  }
}

// spmm.cc:7-25 csr_spmm, faithful: OpenMP over rows, k (output column)
// OUTER and nnz INNER, pattern only (unit values), double dense/out,
// row-major, int64 loop indices. This is the reference CPU baseline.
void oracle_spmm_cc_csr(int64_t num_rows, int64_t num_cols_out, const int64_t* indptr,
                        const int64_t* indices, const double* dense, int64_t dense_cols,
                        double* out) {
#pragma omp parallel for
  for (int64_t rid = 0; rid < num_rows; ++rid) {
    const int64_t row_start = indptr[rid], row_end = indptr[rid + 1];
    double* out_off = out + rid * num_cols_out;
    for (int64_t k = 0; k < num_cols_out; ++k) {
      double acc = 0;
      for (int64_t j = row_start; j < row_end; ++j) acc += dense[indices[j] * dense_cols + k];
      out_off[k] = acc;
    }
  }
}

// spmm.cc:27-43 coo_spmm, faithful: out zeroed (the memset at :32), OpenMP
// over the nnz entries, each adding dense row `col` into out row `row` with
// `omp atomic` (double, unit values). The order of the atomic adds is the
// schedule's, so results can differ from the CSR form in the last bits.
void oracle_spmm_cc_coo(int64_t num_rows, int64_t num_cols_out, int64_t nnz, const int64_t* row,
                        const int64_t* col, const double* dense, int64_t dense_cols, double* out) {
  std::memset(out, 0, sizeof(double) * (size_t)(num_rows * num_cols_out));
#pragma omp parallel for
  for (int64_t i = 0; i < nnz; ++i) {
    const int64_t rid = row[i], cid = col[i];
    double* out_off = out + rid * num_cols_out;
    for (int64_t k = 0; k < num_cols_out; ++k) {
#pragma omp atomic
      out_off[k] += dense[cid * dense_cols + k];
    }
  }
}

// cusparseXcoo2csr semantics (csrmm.cu:148-149): row pointer of a row-sorted
// COO, in the index base of its row indices (csr_rowptr[0] = base,
// csr_rowptr[m] = nnz + base). Restated from the cuSPARSE documentation (the
// library is closed source); pinned by the csrmm.cu KAT, whose rowptr the
// conversion must produce.
void oracle_coo2csr(const int* coo_row, int nnz, int m, int base, int* csr_rowptr) {
  int i = 0;
  for (int r = 0; r <= m; ++r) {
    while (i < nnz && coo_row[i] - base < r) ++i;
    csr_rowptr[r] = i + base;
  }
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

// -------------------------------------------------------------- BSR -----
// cusparseSbsrmm semantics (run_bsrmm.cu:160-165, bsrmm.cu:141-144):
// C = alpha * A_bsr * B + beta * C, A block b stored row-major (dir 0,
// DIRECTION_ROW: val[b*bs*bs + r*bs + c]) or column-major (dir 1). Sum order:
// blocks of the block row in order, k = 0..bs-1 inside a block.
extern "C++" {
template <class T>
static void bsrmm_seq(int dir, int mb, int n, int bs, const int* rowptr, const int* colind,
                      const T* val, const T* B, int ldb, int orderB, T alpha, T beta, T* C,
                      int ldc, int orderC) {
  const size_t bs2 = (size_t)bs * bs;
#pragma omp parallel for schedule(dynamic, 4)
  for (int br = 0; br < mb; ++br) {
    for (int rr = 0; rr < bs; ++rr) {
      const int r = br * bs + rr;
      for (int c = 0; c < n; ++c) {
        T acc = 0;
        for (int k = rowptr[br]; k < rowptr[br + 1]; ++k) {
          const T* blk = val + (size_t)k * bs2;
          for (int q = 0; q < bs; ++q) {
            const T a = dir == 0 ? blk[(size_t)rr * bs + q] : blk[(size_t)q * bs + rr];
            acc = std::fma(a, B[at(colind[k] * bs + q, c, ldb, orderB)], acc);
          }
        }
        T& out = C[at(r, c, ldc, orderC)];
        out = beta == T(0) ? alpha * acc : std::fma(beta, out, alpha * acc);
      }
    }
  }
}
}  // extern "C++"

void oracle_bsrmm_f32(int dir, int mb, int n, int bs, const int* rowptr, const int* colind,
                      const float* val, const float* B, int ldb, int orderB, float alpha,
                      float beta, float* C, int ldc, int orderC) {
  bsrmm_seq<float>(dir, mb, n, bs, rowptr, colind, val, B, ldb, orderB, alpha, beta, C, ldc,
                   orderC);
}

// rocsparse_bsrmm_template<double> (rocsparse_bsrmm.h:102; the double myfma
// overload, rocsparse_bsrmm_impl.h:10).
void oracle_bsrmm_d(int dir, int mb, int n, int bs, const int* rowptr, const int* colind,
                    const double* val, const double* B, int ldb, int orderB, double alpha,
                    double beta, double* C, int ldc, int orderC) {
  bsrmm_seq<double>(dir, mb, n, bs, rowptr, colind, val, B, ldb, orderB, alpha, beta, C, ldc,
                    orderC);
}

// Double-precision BSR product + |a|.|b| (row-major outputs, m = mb*bs rows).
// Values are taken as float or, with half_inputs, as IEEE binary16 patterns.
void oracle_bsrmm_f64(int dir, int mb, int n, int bs, const int* rowptr, const int* colind,
                      const void* val, const void* B, int ldb, int orderB, int half_inputs,
                      double* C, double* absdot) {
  auto h2d = [](uint16_t h) -> double {
    const int s = h >> 15, e = (h >> 10) & 31, f = h & 1023;
    double v;
    if (e == 0) v = std::ldexp((double)f, -24);
    else if (e == 31) v = f ? NAN : INFINITY;
    else v = std::ldexp((double)(f | 1024), e - 25);
    return s ? -v : v;
  };
  auto get = [&](const void* p, size_t i) -> double {
    return half_inputs ? h2d(static_cast<const uint16_t*>(p)[i])
                       : (double)static_cast<const float*>(p)[i];
  };
  const size_t bs2 = (size_t)bs * bs;
#pragma omp parallel for schedule(dynamic, 4)
  for (int br = 0; br < mb; ++br) {
    for (int rr = 0; rr < bs; ++rr) {
      const int r = br * bs + rr;
      for (int c = 0; c < n; ++c) {
        double acc = 0.0, aa = 0.0;
        for (int k = rowptr[br]; k < rowptr[br + 1]; ++k) {
          for (int q = 0; q < bs; ++q) {
            const size_t ai = (size_t)k * bs2 + (dir == 0 ? (size_t)rr * bs + q : (size_t)q * bs + rr);
            const double prod = get(val, ai) * get(B, at(colind[k] * bs + q, c, ldb, orderB));
            acc += prod;
            aa += std::fabs(prod);
          }
        }
        C[(size_t)r * n + c] = acc;
        if (absdot) absdot[(size_t)r * n + c] = aa;
      }
    }
  }
}

// ------------------------------------------------------- conversions -----
// cusparseXcsr2bsrNnz (run_bsrmm.cu:121-131) / calculateNnzb (utility.cc:
// 47-69): block row br's nonzero blocks are the distinct colind/bs of its
// rows, ascending. Restated with std::set (independent of the product's
// marker-array implementation).
int64_t oracle_csr2bsr_nnz(int m, int bs, const int* rowptr, const int* colind, int* bsr_rowptr) {
  const int mb = (m + bs - 1) / bs;
  int64_t acc = 0;
  if (bsr_rowptr) bsr_rowptr[0] = 0;
  for (int br = 0; br < mb; ++br) {
    std::set<int> cols;
    for (int r = br * bs; r < std::min(m, (br + 1) * bs); ++r)
      for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) cols.insert(colind[j] / bs);
    acc += (int64_t)cols.size();
    if (bsr_rowptr) bsr_rowptr[br + 1] = (int)acc;
  }
  return acc;
}

// cusparseScsr2bsr (run_bsrmm.cu:136-142) and divide_matrix at density -> 0
// (divide.cu:52-127, value placement :116): zero-filled blocks, A[r][c] at
// b*bs*bs + (r%bs)*bs + c%bs for DIRECTION_ROW (dir 0), transposed in-block
// for COLUMN. Duplicate (r, c) entries are summed.
void oracle_csr2bsr(int dir, int m, int bs, const int* rowptr, const int* colind,
                    const float* val, const int* bsr_rowptr, int* bsr_colind, float* bsr_val) {
  const int mb = (m + bs - 1) / bs;
  const size_t bs2 = (size_t)bs * bs;
  for (int br = 0; br < mb; ++br) {
    std::map<int, int> slot;
    for (int r = br * bs; r < std::min(m, (br + 1) * bs); ++r)
      for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) slot[colind[j] / bs] = 0;
    int k = bsr_rowptr[br];
    for (auto& kv : slot) {
      kv.second = k;
      bsr_colind[k] = kv.first;
      std::fill(bsr_val + (size_t)k * bs2, bsr_val + (size_t)(k + 1) * bs2, 0.f);
      ++k;
    }
    for (int r = br * bs; r < std::min(m, (br + 1) * bs); ++r) {
      for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
        const int c = colind[j], rr = r - br * bs, cc = c % bs;
        const size_t off = (size_t)slot[c / bs] * bs2 +
                           (dir == 0 ? (size_t)rr * bs + cc : (size_t)cc * bs + rr);
        bsr_val[off] += val[j];
      }
    }
  }
}

// cusparseSbsr2csr (bsr2csr.cu:177-188): every block expanded, zeros kept,
// nnz = nnzb*bs*bs; row r lists, block by block, columns colind[k]*bs + c.
void oracle_bsr2csr(int dir, int mb, int bs, const int* bsr_rowptr, const int* bsr_colind,
                    const float* bsr_val, int* rowptr, int* colind, float* val) {
  const size_t bs2 = (size_t)bs * bs;
  int64_t pos = 0;
  rowptr[0] = 0;
  for (int br = 0; br < mb; ++br)
    for (int rr = 0; rr < bs; ++rr) {
      for (int k = bsr_rowptr[br]; k < bsr_rowptr[br + 1]; ++k)
        for (int c = 0; c < bs; ++c) {
          colind[pos] = bsr_colind[k] * bs + c;
          val[pos] = bsr_val[(size_t)k * bs2 + (dir == 0 ? (size_t)rr * bs + c : (size_t)c * bs + rr)];
          ++pos;
        }
      rowptr[br * bs + rr + 1] = (int)pos;
    }
}

// divide_matrix (divide.cu:52-127) with values: per block row, block column
// bc is admitted to the BSR part iff count(bc)/bs^2 >= density (every column,
// empty ones too, when density <= 0: 0 >= 0). Other entries stay CSR in
// row order. Caller capacities: csr arrays >= nnz, bsr blocks >= cap_blocks.
// out[0] = csr nnz, out[1] = nnzb; returns -1 if a capacity is exceeded.
int oracle_divide(int n, int bs, float density, const int* rowptr, const int* colind,
                  const float* val, int* csr_rp, int* csr_ci, float* csr_v, int* bsr_rp,
                  int* bsr_ci, float* bsr_v, int64_t cap_blocks, int64_t* out) {
  const int nb = (n + bs - 1) / bs;
  const size_t bs2 = (size_t)bs * bs;
  int64_t cpos = 0, bpos = 0;
  csr_rp[0] = 0;
  bsr_rp[0] = 0;
  for (int br = 0; br < nb; ++br) {
    std::map<int, int> cnt;
    const int r0 = br * bs, r1 = std::min(n, r0 + bs);
    for (int r = r0; r < r1; ++r)
      for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) cnt[colind[j] / bs] += 1;
    std::map<int, int64_t> slot;
    for (int bc = 0; bc < nb; ++bc) {
      const auto it = cnt.find(bc);
      const float occupy = (float)((it == cnt.end() ? 0 : it->second) * 1.0 / (double)bs2);
      if (occupy >= density) {
        if (bpos >= cap_blocks) return -1;
        slot[bc] = bpos;
        bsr_ci[bpos] = bc;
        std::fill(bsr_v + bpos * bs2, bsr_v + (bpos + 1) * bs2, 0.f);
        ++bpos;
      }
    }
    bsr_rp[br + 1] = (int)bpos;
    for (int r = r0; r < r1; ++r) {
      for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
        const auto it = slot.find(colind[j] / bs);
        if (it == slot.end()) {
          csr_ci[cpos] = colind[j];
          csr_v[cpos] = val[j];
          ++cpos;
        } else {
          bsr_v[it->second * bs2 + (size_t)(r - r0) * bs + colind[j] % bs] += val[j];
        }
      }
      csr_rp[r + 1] = (int)cpos;
    }
  }
  out[0] = cpos;
  out[1] = bpos;
  return 0;
}

// ---------------------------------------------------------------------------
// Reorder front-end, restated on adjacency lists as the reference holds them.
// kind 0: maxDegreeSort (reorder_strategy.cc:57-71) — descending degree,
//         std::sort on (id, degree) records in id order (unstable, as there);
// kind 1: BFSTraversal (:84-114) — FIFO over adjacency order, the smallest
//         unvisited id starts each component;
// kind 2: reverseCuthillMcKee (:73-82) — every list std::sort-ed by
//         descending degree, then kind 1 (no final reversal, as there);
// kind 3: permutate(old2new) (:42-55) — rename, move rows, sort lists.
// Output: the reordered graph as CSR (out_rowptr[n+1], out_colind[nnz]).
int oracle_reorder(int kind, int n, const int* rowptr, const int* colind, const int* perm,
                   int* out_rowptr, int* out_colind) {
  std::vector<std::vector<int>> e(n);
  for (int i = 0; i < n; ++i) e[i].assign(colind + rowptr[i], colind + rowptr[i + 1]);
  std::vector<int> old2new(n, -1);
  if (kind == 0) {
    std::vector<std::pair<int, int>> nodes;  // (id, degree)
    for (int i = 0; i < n; ++i) nodes.emplace_back(i, (int)e[i].size());
    std::sort(nodes.begin(), nodes.end(),
              [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
                return a.second > b.second;
              });
    for (int i = 0; i < n; ++i) old2new[nodes[i].first] = i;
  } else if (kind == 1 || kind == 2) {
    if (kind == 2)
      for (auto& l : e)
        std::sort(l.begin(), l.end(), [&e](int x, int y) { return e[x].size() > e[y].size(); });
    int cnt = 0;
    for (int root = 0; root < n; ++root) {
      if (old2new[root] != -1) continue;
      std::vector<int> q{root};
      old2new[root] = cnt++;
      for (size_t h = 0; h < q.size(); ++h)
        for (int y : e[q[h]])
          if (old2new[y] == -1) {
            old2new[y] = cnt++;
            q.push_back(y);
          }
    }
  } else if (kind == 3) {
    old2new.assign(perm, perm + n);
  } else {
    return -1;
  }
  std::vector<std::vector<int>> ne(n);
  for (int i = 0; i < n; ++i) {
    for (int& c : e[i]) c = old2new[c];
    ne[old2new[i]] = std::move(e[i]);
  }
  out_rowptr[0] = 0;
  for (int i = 0; i < n; ++i) {
    std::sort(ne[i].begin(), ne[i].end());
    std::copy(ne[i].begin(), ne[i].end(), out_colind + out_rowptr[i]);
    out_rowptr[i + 1] = out_rowptr[i] + (int)ne[i].size();
  }
  return 0;
}

}  // extern "C"

