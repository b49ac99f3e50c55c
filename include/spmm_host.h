/*
 * spmm_host.h — host data feeders of libspmm_hip.so.
 *
 * C restatements of the reference's load_data.h / utility.h host helpers so
 * the drivers (run_csrmm, run_bsrmm, test_csrmm, test_bsrmm) and bench.py can
 * produce exactly the reference's inputs:
 *   randomArray / randomDenseMatrix   load_data.cc:29-40  (mt19937_64 seeded 1234,
 *                                      uniform_real_distribution<float>)
 *   randomCSRMatrix                   load_data.cc:42-69
 *   randomBSRMatrix                   load_data.cc:81-113
 *   dumpCSRToFile / loadCSRFromFile   load_data.cc:125-165 (text CSR format)
 *   loadGraphFromFile                 load_data.cc:167-184 ("n nnz" + edge list)
 * (text parsed and written by worker threads, host_io.cpp; same results as the
 * reference's iostream loops on well-formed files, -1 on malformed ones)
 * All of them draw from ONE process-wide generator, as the reference's
 * `static std::mt19937_64 gen(1234)` (load_data.cc:12) does, so call order
 * matters exactly as it does there. Arrays returned through T** are
 * malloc'ed; release them with spmm_host_free.
 *
 * Plus synthetic stand-ins for the absent OGB / reddit datasets (no network):
 *   spmm_host_gen_powerlaw_csr     Chung-Lu power-law graph (ogbn-arxiv/products)
 *   spmm_host_gen_community_csr    community-structured graph in community
 *                                  order (stand-in for a rabbit-reordered reddit)
 */
#ifndef SPMM_HOST_H
#define SPMM_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void spmm_host_free(void* p);

/* Reset the shared generator (the reference seeds it once with 1234). */
void spmm_host_rng_seed(uint64_t seed);

/* randomArray(n, minVal, maxVal) into caller memory. */
void spmm_host_random_array(int64_t n, float minVal, float maxVal, float* out);

/* randomCSRMatrix(m, n, p, ...): Bernoulli(p) per (row, col) in row-major
 * order, value drawn right after each hit. rowptr has m+1 entries (caller
 * memory); colind / val are malloc'ed. Returns nnz (or -1). */
int64_t spmm_host_random_csr(int m, int n, float p, float minVal, float maxVal, int* rowptr,
                             int** colind, float** val);

/* randomBSRMatrix(mb, nb, blockDim, p, ...): per hit, bs*bs values. */
int64_t spmm_host_random_bsr(int mb, int nb, int blockDim, float p, float minVal, float maxVal,
                             int* rowptr, int** colind, float** val);

/* Text CSR files <prefix>_indptr.txt / <prefix>_indices.txt. */
int spmm_host_dump_csr(const char* prefix, int n, int64_t nnz, const int* rowptr,
                       const int* colind);
int spmm_host_load_csr(const char* prefix, int** rowptr, int** colind, int* n, int64_t* nnz);

/* Edge list "n nnz\n src dst ..." -> CSR with sorted neighbours (duplicates
 * kept, as in the reference). Returns 0 on success. */
int spmm_host_load_graph(const char* filename, int** rowptr, int** colind, int* n, int64_t* nnz);

/* Binary sidecar cache: header (magic "SPMMCSR1",
 * version, flags, n, nnz, one 64-bit checksum per array) + rowptr[n+1] +
 * colind[nnz] (+ val[nnz] when given). Written under a temporary name and
 * renamed. load returns 0, -1 (missing / not a cache / I/O error) or -2
 * (checksum mismatch: the file is corrupt). *val is NULL when the file has no
 * values; pass val = NULL to ignore them. */
int spmm_host_save_csr_bin(const char* path, int n, int64_t nnz, const int* rowptr,
                           const int* colind, const float* val);
int spmm_host_load_csr_bin(const char* path, int** rowptr, int** colind, float** val, int* n,
                           int64_t* nnz);

/* loadCSRFromFile through the cache: <prefix>.csrbin is used when it is at
 * least as new as both text files and intact; otherwise the text is parsed
 * and the cache (re)written. The text format is unchanged. */
int spmm_host_load_csr_cached(const char* prefix, int** rowptr, int** colind, int* n,
                              int64_t* nnz);

/* Chung-Lu power-law digraph: expected degree w_i = c*(i+s)^(-1/(gamma-1)),
 * w_0 = max_deg, sum w = nnz_target; row i draws d_i distinct columns with
 * probability proportional to w_j; node ids are then randomly relabelled.
 * Deterministic in (n, nnz_target, max_deg, gamma, seed), independent of the
 * thread count. Exactly nnz_target nonzeros, sorted columns, no duplicates. */
int spmm_host_gen_powerlaw_csr(int n, int64_t nnz_target, int max_deg, double gamma,
                               uint64_t seed, int** rowptr, int** colind);

/* Community graph: nodes 0..n-1 split into contiguous communities with sizes
 * drawn from [cmin, cmax]; each row has `avg_deg` expected out-edges, a
 * fraction p_in inside its own community (uniform), the rest uniform over
 * all nodes. Node order is the community order (what a community reordering
 * such as rabbit_order recovers). Returns 0 on success; *nnz_out is set. */
int spmm_host_gen_community_csr(int n, double avg_deg, int cmin, int cmax, double p_in,
                                uint64_t seed, int** rowptr, int** colind, int64_t* nnz_out);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_HOST_H */
