// reorder.cpp — reorder-aware preprocessing front-end (include/spmm_reorder.h).
//
// Works on CSR arrays directly (the reference holds vector<vector<int>>
// adjacency lists, reorder_strategy.cc); per-row work runs on worker threads,
// the BFS itself is sequential (its visit order is the result).
#include "spmm_reorder.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <numeric>
#include <string>
#include <vector>

#include "host_util.hpp"

using spmm_host::parallel_for;

namespace {

bool valid_csr(int n, const int* rowptr, const int* colind) {
  if (n < 0 || (n > 0 && !rowptr)) return false;
  if (n == 0) return true;
  if (rowptr[0] != 0) return false;
  for (int i = 0; i < n; ++i)
    if (rowptr[i + 1] < rowptr[i]) return false;
  if (rowptr[n] > 0 && !colind) return false;
  std::atomic<bool> ok{true};
  parallel_for(rowptr[n], [&](int64_t lo, int64_t hi) {
    for (int64_t j = lo; j < hi; ++j)
      if (colind[j] < 0 || colind[j] >= n) {
        ok = false;
        return;
      }
  });
  return ok.load();
}

// BFS visit order (BFSTraversal, reorder_strategy.cc:84-114) over the
// adjacency lists adj[rowptr[x] .. rowptr[x+1]) in their given order.
void bfs_order(int n, const int* rowptr, const int* adj, int* old2new) {
  std::fill(old2new, old2new + n, -1);
  std::vector<int> queue(n);
  int cnt = 0, pos = 0;
  while (true) {
    // The next unvisited node with the smallest id starts a component.
    for (; pos < n && old2new[pos] != -1; ++pos) {
    }
    if (pos == n) break;
    int head = 0, tail = 0;
    old2new[pos] = cnt++;
    queue[tail++] = pos;
    while (head < tail) {
      const int x = queue[head++];
      for (int j = rowptr[x]; j < rowptr[x + 1]; ++j) {
        const int y = adj[j];
        if (old2new[y] == -1) {
          old2new[y] = cnt++;
          queue[tail++] = y;
        }
      }
    }
  }
}

}  // namespace

extern "C" {

int spmm_check_permutation(int n, const int* old2new) {
  if (n < 0 || (n > 0 && !old2new)) return -1;
  std::vector<char> seen(n, 0);
  for (int i = 0; i < n; ++i) {
    const int v = old2new[i];
    if (v < 0 || v >= n || seen[v]) return -1;
    seen[v] = 1;
  }
  return 0;
}

int spmm_reorder_degree(int n, const int* rowptr, const int* colind, int* old2new) {
  if (!valid_csr(n, rowptr, colind) || (n > 0 && !old2new)) return -1;
  struct Node {
    int id, val;
  };
  std::vector<Node> nodes(n);
  for (int i = 0; i < n; ++i) nodes[i] = {i, rowptr[i + 1] - rowptr[i]};
  // Unstable on purpose: equal degrees land where libstdc++'s introsort puts
  // them, exactly as in maxDegreeSort (reorder_strategy.cc:63-65).
  std::sort(nodes.begin(), nodes.end(), [](const Node& a, const Node& b) { return a.val > b.val; });
  for (int i = 0; i < n; ++i) old2new[nodes[i].id] = i;
  return 0;
}

int spmm_reorder_bfs(int n, const int* rowptr, const int* colind, int* old2new) {
  if (!valid_csr(n, rowptr, colind) || (n > 0 && !old2new)) return -1;
  bfs_order(n, rowptr, colind, old2new);
  return 0;
}

int spmm_reorder_rcm(int n, const int* rowptr, const int* colind, int* old2new) {
  if (!valid_csr(n, rowptr, colind) || (n > 0 && !old2new)) return -1;
  const int64_t nnz = n ? rowptr[n] : 0;
  std::vector<int> adj(colind, colind + nnz);
  // Each list by descending degree (reorder_strategy.cc:75-80); rows are
  // independent, so the per-row unstable sorts run in parallel unchanged.
  parallel_for(n, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i)
      std::sort(adj.begin() + rowptr[i], adj.begin() + rowptr[i + 1], [&](int x, int y) {
        return rowptr[x + 1] - rowptr[x] > rowptr[y + 1] - rowptr[y];
      });
  });
  bfs_order(n, rowptr, adj.data(), old2new);
  return 0;
}

int spmm_permute_csr(int n, const int* rowptr, const int* colind, const float* val,
                     const int* old2new, int* new_rowptr, int* new_colind, float* new_val) {
  if (!valid_csr(n, rowptr, colind) || !new_rowptr || (!val) != (!new_val)) return -1;
  if (spmm_check_permutation(n, old2new) != 0) return -1;
  const int64_t nnz = n ? rowptr[n] : 0;
  if (nnz > 0 && !new_colind) return -1;
  new_rowptr[0] = 0;
  {
    std::vector<int> deg(n);
    for (int i = 0; i < n; ++i) deg[old2new[i]] = rowptr[i + 1] - rowptr[i];
    for (int i = 0; i < n; ++i) new_rowptr[i + 1] = new_rowptr[i] + deg[i];
  }
  parallel_for(n, [&](int64_t lo, int64_t hi) {
    std::vector<std::pair<int, int>> tmp;  // (new column, source position)
    for (int64_t i = lo; i < hi; ++i) {
      const int dst = new_rowptr[old2new[i]];
      const int b = rowptr[i], e = rowptr[i + 1];
      if (!val) {
        for (int j = b; j < e; ++j) new_colind[dst + j - b] = old2new[colind[j]];
        std::sort(new_colind + dst, new_colind + dst + (e - b));
        continue;
      }
      tmp.resize(e - b);
      for (int j = b; j < e; ++j) tmp[j - b] = {old2new[colind[j]], j};
      std::sort(tmp.begin(), tmp.end());  // ties by source position: stable
      for (int t = 0; t < e - b; ++t) {
        new_colind[dst + t] = tmp[t].first;
        new_val[dst + t] = val[tmp[t].second];
      }
    }
  });
  return 0;
}

int spmm_load_permutation(const char* filename, int n, int* old2new) {
  if (!filename || n < 0 || (n > 0 && !old2new)) return -1;
  FILE* f = std::fopen(filename, "r");
  if (!f) return -1;
  int i = 0;
  for (; i < n; ++i)
    if (std::fscanf(f, "%d", &old2new[i]) != 1) break;
  std::fclose(f);
  if (i != n) return -1;
  return spmm_check_permutation(n, old2new);
}

int spmm_dump_permutation(const char* filename, int n, const int* old2new) {
  if (!filename || spmm_check_permutation(n, old2new) != 0) return -1;
  FILE* f = std::fopen(filename, "w");
  if (!f) return -1;
  for (int i = 0; i < n; ++i) std::fprintf(f, "%d\n", old2new[i]);
  return std::fclose(f) == 0 ? 0 : -1;
}

int spmm_block_metrics(int n, const int* rowptr, const int* colind, int blockDim,
                       spmm_block_metrics_t* out) {
  if (!valid_csr(n, rowptr, colind) || blockDim <= 0 || !out) return -1;
  const int nb = (n + blockDim - 1) / blockDim;
  const int64_t nnz = n ? rowptr[n] : 0;
  std::vector<int64_t> per(nb, 0);
  parallel_for(nb, [&](int64_t lo, int64_t hi) {
    std::vector<int> mark(nb, -1);
    for (int64_t br = lo; br < hi; ++br) {
      int64_t c = 0;
      const int r1 = (int)std::min<int64_t>(n, (br + 1) * blockDim);
      for (int r = (int)(br * blockDim); r < r1; ++r)
        for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
          const int bc = colind[j] / blockDim;
          if (mark[bc] != br) {
            mark[bc] = (int)br;
            ++c;
          }
        }
      per[br] = c;
    }
  });
  const int64_t nnzb = std::accumulate(per.begin(), per.end(), (int64_t)0);
  const double bs = blockDim;
  out->block_dim = blockDim;
  out->nnzb = nnzb;
  out->density = nb ? (double)nnzb / ((double)nb * (double)nb) : 0.0;
  out->utilization = nnzb ? (double)nnz / ((double)nnzb * bs * bs) : 0.0;
  out->average = nnzb ? (double)nnz / (double)nnzb : 0.0;
  return 0;
}

int spmm_block_heatmap(int n, const int* rowptr, const int* colind, int blockDim, int* heatmap) {
  if (!valid_csr(n, rowptr, colind) || blockDim <= 0) return -1;
  const int64_t nb = (n + blockDim - 1) / blockDim;
  if (nb > 0 && !heatmap) return -1;
  parallel_for(nb, [&](int64_t lo, int64_t hi) {
    for (int64_t br = lo; br < hi; ++br) {
      int* row = heatmap + br * nb;
      std::fill(row, row + nb, 0);
      const int r1 = (int)std::min<int64_t>(n, (br + 1) * blockDim);
      for (int r = (int)(br * blockDim); r < r1; ++r)
        for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) ++row[colind[j] / blockDim];
    }
  });
  return 0;
}

int spmm_dump_heatmap(const char* filename, int nb, const int* heatmap) {
  if (!filename || nb <= 0 || !heatmap) return -1;
  std::ofstream fs(filename);
  if (!fs) return -1;
  fs << nb << '\n';
  std::string line;
  char buf[16];
  for (int64_t i = 0; i < nb; ++i) {
    line.clear();
    for (int64_t j = 0; j < nb; ++j) {
      const int len = std::snprintf(buf, sizeof buf, "%d ", heatmap[i * nb + j]);
      line.append(buf, len);
    }
    line.push_back('\n');
    fs << line;
  }
  return fs.good() ? 0 : -1;
}

}  // extern "C"
