// host_data.cpp — host data feeders and synthetic graph generators
// (declared in include/spmm_host.h; see there for the reference mapping).
#include "spmm_host.h"

#include "host_util.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

// The reference keeps one generator for the whole process (load_data.cc:12).
std::mt19937_64& shared_gen() {
  static std::mt19937_64 gen(1234);
  return gen;
}
std::mutex& gen_mu() {
  static std::mutex mu;
  return mu;
}

template <typename T>
T* to_malloc(const std::vector<T>& v) {
  T* p = static_cast<T*>(std::malloc(std::max<size_t>(1, v.size()) * sizeof(T)));
  if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

using spmm_host::num_threads;
using spmm_host::parallel_for;

// Vose alias table over weights w.
struct Alias {
  std::vector<double> prob;
  std::vector<int> alias;
  explicit Alias(const std::vector<double>& w) {
    const int n = (int)w.size();
    prob.assign(n, 0.0);
    alias.assign(n, 0);
    const double sum = std::accumulate(w.begin(), w.end(), 0.0);
    std::vector<double> q(n);
    std::vector<int> small, large;
    for (int i = 0; i < n; ++i) {
      q[i] = w[i] * n / sum;
      (q[i] < 1.0 ? small : large).push_back(i);
    }
    while (!small.empty() && !large.empty()) {
      const int s = small.back(), l = large.back();
      small.pop_back();
      prob[s] = q[s];
      alias[s] = l;
      q[l] = (q[l] + q[s]) - 1.0;
      if (q[l] < 1.0) {
        large.pop_back();
        small.push_back(l);
      }
    }
    for (int l : large) prob[l] = 1.0;
    for (int s : small) prob[s] = 1.0;
  }
  template <typename G>
  int sample(G& g) const {
    const uint64_t r = g();
    const int i = (int)((r >> 11) % prob.size());
    const double u = (double)(g() >> 11) * (1.0 / 9007199254740992.0);
    return u < prob[i] ? i : alias[i];
  }
};

// Per-row draw of `d` distinct values from `alias`, sorted.
template <typename G>
void draw_distinct(const Alias& a, int d, G& g, std::vector<int>& out) {
  out.clear();
  while ((int)out.size() < d) {
    const int need = d - (int)out.size();
    for (int t = 0; t < need; ++t) out.push_back(a.sample(g));
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
  }
}

}  // namespace

extern "C" {

void spmm_host_free(void* p) { std::free(p); }

void spmm_host_rng_seed(uint64_t seed) {
  std::lock_guard<std::mutex> lk(gen_mu());
  shared_gen().seed(seed);
}

void spmm_host_random_array(int64_t n, float minVal, float maxVal, float* out) {
  std::lock_guard<std::mutex> lk(gen_mu());
  std::uniform_real_distribution<float> dist(minVal, maxVal);
  auto& g = shared_gen();
  for (int64_t i = 0; i < n; ++i) out[i] = dist(g);
}

int64_t spmm_host_random_csr(int m, int n, float p, float minVal, float maxVal, int* rowptr,
                             int** colind, float** val) {
  if (m < 0 || n < 0 || !rowptr || !colind || !val) return -1;
  std::lock_guard<std::mutex> lk(gen_mu());
  std::uniform_real_distribution<float> flip(0, 1), dist(minVal, maxVal);
  auto& g = shared_gen();
  std::vector<int> idx;
  std::vector<float> vals;
  int64_t cnt = 0;
  rowptr[0] = 0;
  for (int i = 1; i <= m; ++i) {
    for (int j = 0; j < n; ++j) {
      if (flip(g) < p) {
        idx.push_back(j);
        vals.push_back(dist(g));
        ++cnt;
      }
    }
    rowptr[i] = (int)cnt;
  }
  *colind = to_malloc(idx);
  *val = to_malloc(vals);
  return cnt;
}

int64_t spmm_host_random_bsr(int mb, int nb, int blockDim, float p, float minVal, float maxVal,
                             int* rowptr, int** colind, float** val) {
  if (mb < 0 || nb < 0 || blockDim <= 0 || !rowptr || !colind || !val) return -1;
  std::lock_guard<std::mutex> lk(gen_mu());
  std::uniform_real_distribution<float> flip(0, 1), dist(minVal, maxVal);
  auto& g = shared_gen();
  const int bnum = blockDim * blockDim;
  std::vector<int> idx;
  std::vector<float> vals;
  int64_t cnt = 0;
  rowptr[0] = 0;
  for (int i = 1; i <= mb; ++i) {
    for (int j = 0; j < nb; ++j) {
      if (flip(g) < p) {
        idx.push_back(j);
        for (int k = 0; k < bnum; ++k) vals.push_back(dist(g));
        ++cnt;
      }
    }
    rowptr[i] = (int)cnt;
  }
  *colind = to_malloc(idx);
  *val = to_malloc(vals);
  return cnt;
}

// spmm_host_dump_csr / spmm_host_load_csr / spmm_host_load_graph: host_io.cpp.

int spmm_host_gen_powerlaw_csr(int n, int64_t nnz_target, int max_deg, double gamma,
                               uint64_t seed, int** rowptr_out, int** colind_out) {
  if (n <= 0 || nnz_target < 0 || max_deg <= 0 || gamma <= 1.0 || !rowptr_out || !colind_out)
    return -1;
  if ((double)max_deg > 0.5 * n || nnz_target > (int64_t)n * (n / 2) || nnz_target > INT32_MAX)
    return -1;
  const double beta = 1.0 / (gamma - 1.0);
  // Solve the offset s so that sum_i max_deg * ((i + s) / s)^(-beta) = nnz.
  // Exact over the steep head, strided over the tail (s only needs to be
  // approximate: degrees are rescaled to hit nnz_target exactly below).
  auto total_for = [&](double s) {
    double t = 0.0;
    const int head = std::min(n, 4096);
    for (int i = 0; i < head; ++i) t += std::pow((i + s) / s, -beta);
    const int st = std::max(1, (n - head) / 65536);
    for (int i = head; i < n; i += st) t += std::pow((i + s) / s, -beta) * std::min(st, n - i);
    return t * max_deg;
  };
  double lo = 1e-3, hi = 1e9;
  for (int it = 0; it < 80 && hi / lo > 1.0 + 1e-9; ++it) {
    const double mid = std::sqrt(lo * hi);
    if (total_for(mid) < (double)nnz_target) lo = mid; else hi = mid;
  }
  const double s = std::sqrt(lo * hi);
  std::vector<double> w(n);
  for (int i = 0; i < n; ++i) w[i] = max_deg * std::pow((i + s) / s, -beta);
  // Integer degrees summing exactly to nnz_target (cumulative rounding).
  const double wsum = std::accumulate(w.begin(), w.end(), 0.0);
  std::vector<int> deg(n);
  double cum = 0.0;
  int64_t prev = 0;
  for (int i = 0; i < n; ++i) {
    cum += w[i];
    int64_t cur = (int64_t)std::llround(cum / wsum * (double)nnz_target);
    if (i == n - 1) cur = nnz_target;
    deg[i] = (int)std::min<int64_t>(cur - prev, n / 2);
    prev += deg[i];
  }
  // Deficit from the n/2 cap (never hit at the configured sizes) goes to row n-1.
  deg[n - 1] += (int)(nnz_target - prev);
  const Alias alias(w);
  // Random relabelling of node ids (hubs scattered over the id space).
  std::vector<int> perm(n);
  std::iota(perm.begin(), perm.end(), 0);
  {
    std::mt19937_64 g(splitmix64(seed ^ 0xA5A5A5A5ull));
    for (int i = n - 1; i > 0; --i) {
      const int j = (int)(g() % (uint64_t)(i + 1));
      std::swap(perm[i], perm[j]);
    }
  }
  // Row r of the output is generator row inv[r] (perm maps generator -> output).
  std::vector<int> inv(n);
  for (int i = 0; i < n; ++i) inv[perm[i]] = i;
  std::vector<int> rp(n + 1, 0);
  for (int r = 0; r < n; ++r) rp[r + 1] = rp[r] + deg[inv[r]];
  int* ci = static_cast<int*>(std::malloc(sizeof(int) * (size_t)std::max<int64_t>(1, nnz_target)));
  if (!ci) return -1;
  parallel_for(n, [&](int64_t lo_r, int64_t hi_r) {
    std::vector<int> cols;
    for (int64_t r = lo_r; r < hi_r; ++r) {
      const int gi = inv[r];
      std::mt19937_64 g(splitmix64(seed * 0x100000001B3ull + (uint64_t)gi));
      draw_distinct(alias, deg[gi], g, cols);
      for (int& c : cols) c = perm[c];
      std::sort(cols.begin(), cols.end());
      std::copy(cols.begin(), cols.end(), ci + rp[r]);
    }
  });
  *rowptr_out = to_malloc(rp);
  *colind_out = ci;
  return 0;
}

int spmm_host_gen_community_csr(int n, double avg_deg, int cmin, int cmax, double p_in,
                                uint64_t seed, int** rowptr_out, int** colind_out,
                                int64_t* nnz_out) {
  if (n <= 0 || avg_deg < 0 || cmin <= 0 || cmax < cmin || p_in < 0 || p_in > 1 ||
      !rowptr_out || !colind_out || !nnz_out)
    return -1;
  // Contiguous communities with log-uniform sizes in [cmin, cmax].
  std::vector<int> cstart;
  {
    std::mt19937_64 g(splitmix64(seed ^ 0xC0FFEEull));
    std::uniform_real_distribution<double> u(std::log((double)cmin), std::log((double)cmax + 1));
    int pos = 0;
    while (pos < n) {
      cstart.push_back(pos);
      pos += std::max(1, (int)std::exp(u(g)));
    }
    cstart.push_back(n);
  }
  std::vector<int> comm_of(n);
  for (size_t c = 0; c + 1 < cstart.size(); ++c)
    for (int i = cstart[c]; i < cstart[c + 1]; ++i) comm_of[i] = (int)c;
  std::vector<std::vector<int>> rows(n);
  parallel_for(n, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      std::mt19937_64 g(splitmix64(seed * 131 + (uint64_t)r));
      std::uniform_real_distribution<double> u(0.5, 1.5);
      const int c = comm_of[r];
      const int c0 = cstart[c], csz = cstart[c + 1] - c0;
      const double d = avg_deg * u(g);
      const int din = std::min(csz, (int)std::lround(d * p_in));
      const int dout = std::min(n / 2, (int)std::lround(d * (1 - p_in)));
      std::vector<int>& cols = rows[r];
      cols.reserve(din + dout);
      for (int t = 0; t < din; ++t) cols.push_back(c0 + (int)(g() % (uint64_t)csz));
      for (int t = 0; t < dout; ++t) cols.push_back((int)(g() % (uint64_t)n));
      std::sort(cols.begin(), cols.end());
      cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    }
  });
  std::vector<int> rp(n + 1, 0);
  for (int r = 0; r < n; ++r) rp[r + 1] = rp[r] + (int)rows[r].size();
  const int64_t nnz = rp[n];
  int* ci = static_cast<int*>(std::malloc(sizeof(int) * (size_t)std::max<int64_t>(1, nnz)));
  if (!ci) return -1;
  parallel_for(n, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      std::copy(rows[r].begin(), rows[r].end(), ci + rp[r]);
      std::vector<int>().swap(rows[r]);
    }
  });
  *rowptr_out = to_malloc(rp);
  *colind_out = ci;
  *nnz_out = nnz;
  return 0;
}

}  // extern "C"
