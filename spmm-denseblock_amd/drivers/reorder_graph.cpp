// reorder_graph <dataset> [method]  — the reference's reorder_graph CLI
// (reorder_graph.cc:26-48) on the library's reorder front-end.
//
// Reads tmp/<dataset>.txt ("n nnz" + edge list, load_data.cc:167-184), then
// for the original order and for the reordered graph writes
//   tmp/<dataset>_<tag>_indptr.txt / _indices.txt   (CSR text, load_data.cc:125-141)
//   tmp/<dataset>_<tag>_heatmap.txt                 (256 x 256 blocks, utility.cc:90-100)
// and prints analyzeBlockSparseMetrics' lines (reorder_graph.cc:12-24).
// method: rcm (default, tag "rcmk" as in the reference), bfs, degree.
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

#include "spmm_host.h"
#include "spmm_reorder.h"

static void die(const std::string& what) {
  std::cout << what << std::endl;
  std::exit(-1);
}

static void emit(const std::string& prefix, int n, int64_t nnz, const int* rp, const int* ci) {
  if (spmm_host_dump_csr(prefix.c_str(), n, nnz, rp, ci) != 0) die("cannot write " + prefix);
  for (int bs : {2, 4, 8, 16, 32, 64}) {
    spmm_block_metrics_t m;
    if (spmm_block_metrics(n, rp, ci, bs, &m) != 0) die("block metrics failed");
    std::cout << "blockSize=" << bs << " density=" << m.density
              << " utilization=" << m.utilization << " average=" << m.average << std::endl;
  }
  const int nb = (n + 255) / 256;
  std::vector<int> heat((size_t)nb * nb);
  if (spmm_block_heatmap(n, rp, ci, 256, heat.data()) != 0 ||
      spmm_dump_heatmap((prefix + "_heatmap.txt").c_str(), nb, heat.data()) != 0)
    die("cannot write " + prefix + "_heatmap.txt");
}

int main(int argc, char* argv[]) {
  if (argc < 2) die("usage: reorder_graph <dataset> [rcm|bfs|degree]");
  const std::string dataset = argv[1];
  const std::string method = argc > 2 ? argv[2] : "rcm";
  std::cout << "dataset=" << dataset << std::endl;
  int *rp = nullptr, *ci = nullptr, n = 0;
  int64_t nnz = 0;
  if (spmm_host_load_graph(("tmp/" + dataset + ".txt").c_str(), &rp, &ci, &n, &nnz) != 0)
    die("cannot read tmp/" + dataset + ".txt");
  std::cout << "n=" << n << " nnz=" << nnz << std::endl;
  emit("tmp/" + dataset + "_original", n, nnz, rp, ci);

  std::vector<int> old2new(n);
  int rc;
  std::string tag;
  if (method == "rcm") {
    rc = spmm_reorder_rcm(n, rp, ci, old2new.data());
    tag = "rcmk";
  } else if (method == "bfs") {
    rc = spmm_reorder_bfs(n, rp, ci, old2new.data());
    tag = "bfs";
  } else if (method == "degree") {
    rc = spmm_reorder_degree(n, rp, ci, old2new.data());
    tag = "degree";
  } else {
    die("unknown method " + method);
  }
  if (rc != 0) die("reorder failed");
  std::vector<int> nrp(n + 1), nci(nnz);
  if (spmm_permute_csr(n, rp, ci, nullptr, old2new.data(), nrp.data(), nci.data(), nullptr) != 0)
    die("permute failed");
  emit("tmp/" + dataset + "_" + tag, n, nnz, nrp.data(), nci.data());
  spmm_host_free(rp);
  spmm_host_free(ci);
  return 0;
}
