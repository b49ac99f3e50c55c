// rabbit_reorder <dataset>  — the reference's permutation-ingest CLI
// (rabbit_reorder.cc:21-34): applies an external old2new permutation
// (rabbit_order / Gorder output, tmp/<dataset>_rabbit.txt) to
// tmp/<dataset>.txt and writes the CSR text files tmp/<dataset>_rabbit_*.
// The permutation is validated (the reference trusts it).
#include <iostream>
#include <string>
#include <vector>

#include "spmm_host.h"
#include "spmm_reorder.h"

int main(int argc, char* argv[]) {
  if (argc < 2) {
    std::cout << "usage: rabbit_reorder <dataset>" << std::endl;
    return -1;
  }
  const std::string dataset = argv[1];
  std::cout << "dataset=" << dataset << std::endl;
  int *rp = nullptr, *ci = nullptr, n = 0;
  int64_t nnz = 0;
  if (spmm_host_load_graph(("tmp/" + dataset + ".txt").c_str(), &rp, &ci, &n, &nnz) != 0) {
    std::cout << "cannot read tmp/" << dataset << ".txt" << std::endl;
    return -1;
  }
  std::cout << "n=" << n << " nnz=" << nnz << std::endl;
  std::vector<int> old2new(n);
  if (spmm_load_permutation(("tmp/" + dataset + "_rabbit.txt").c_str(), n, old2new.data()) != 0) {
    std::cout << "tmp/" << dataset << "_rabbit.txt is missing or not a permutation of " << n
              << std::endl;
    return -1;
  }
  std::vector<int> nrp(n + 1), nci(nnz);
  if (spmm_permute_csr(n, rp, ci, nullptr, old2new.data(), nrp.data(), nci.data(), nullptr) != 0 ||
      spmm_host_dump_csr(("tmp/" + dataset + "_rabbit").c_str(), n, nnz, nrp.data(), nci.data()) != 0) {
    std::cout << "writing tmp/" << dataset << "_rabbit failed" << std::endl;
    return -1;
  }
  spmm_host_free(rp);
  spmm_host_free(ci);
  return 0;
}
