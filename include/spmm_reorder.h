/*
 * spmm_reorder.h — reorder-aware preprocessing front-end of libspmm_hip.so
 * (SURVEY.md §8f rank 2). Host C++, multi-threaded where the reference's
 * result allows it; the reorder itself stays on the CPU (north_star).
 *
 * A permutation is `old2new` (new id of old node i), the convention of the
 * reference's permutate() and of the rabbit_order / Gorder permutation files.
 *
 *   spmm_reorder_degree     maxDegreeSort            reorder_strategy.cc:57-71
 *   spmm_reorder_bfs        BFSTraversal             reorder_strategy.cc:84-114
 *   spmm_reorder_rcm        reverseCuthillMcKee      reorder_strategy.cc:73-82
 *   spmm_permute_csr        permutate (+ values)     reorder_strategy.cc:42-55
 *   spmm_load_permutation   loadPermutation          rabbit_reorder.cc:10-19
 *   spmm_block_metrics      analyzeBlockSparseMetrics reorder_graph.cc:12-24
 *   spmm_block_heatmap      getHeatmap               utility.cc:71-88
 *   spmm_dump_heatmap       dumpHeatmap              utility.cc:90-100
 *
 * Tie order: maxDegreeSort and the neighbour ordering inside
 * reverseCuthillMcKee use an unstable std::sort in the reference, so nodes of
 * equal degree come out in the order libstdc++'s introsort leaves them. The
 * functions here apply the same comparator to the same input sequence with
 * the same library, so their output is bit-identical to the reference's
 * (checked against the reference's own reorder_strategy.cc in
 * tests/test_reorder.py).
 *
 * All functions return 0 on success and -1 on invalid input (null pointers,
 * negative sizes, column ids out of range, a non-permutation, I/O failure).
 */
#ifndef SPMM_REORDER_H
#define SPMM_REORDER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Descending out-degree order (ties: libstdc++ std::sort, as the reference). */
int spmm_reorder_degree(int n, const int* rowptr, const int* colind, int* old2new);

/* Breadth-first order over out-edges in adjacency order; every unvisited
 * node with the smallest id starts a new component. */
int spmm_reorder_bfs(int n, const int* rowptr, const int* colind, int* old2new);

/* The reference's "reverseCuthillMcKee": each adjacency list re-sorted by
 * descending degree, then the BFS order above (no final reversal — the
 * reference does not reverse it). */
int spmm_reorder_rcm(int n, const int* rowptr, const int* colind, int* old2new);

/* Symmetric permutation: row old2new[i] of the output holds row i with every
 * column c renamed old2new[c], columns sorted ascending (values follow their
 * columns; equal columns keep their input order). new_rowptr has n+1
 * entries, new_colind / new_val nnz. val / new_val may both be NULL. */
int spmm_permute_csr(int n, const int* rowptr, const int* colind, const float* val,
                     const int* old2new, int* new_rowptr, int* new_colind, float* new_val);

/* 0 if old2new is a permutation of [0, n), else -1. */
int spmm_check_permutation(int n, const int* old2new);

/* Text permutation file: n whitespace-separated old2new entries (the format
 * rabbit_order's demo and Gorder write). Validated as a permutation. */
int spmm_load_permutation(const char* filename, int n, int* old2new);
int spmm_dump_permutation(const char* filename, int n, const int* old2new);

/* Block statistics of the pattern at one block size, as printed by
 * analyzeBlockSparseMetrics: density = nnzb / nb^2, utilization =
 * nnz / (nnzb * bs^2), average = nnz / nnzb (nb = ceil(n / bs)). */
typedef struct {
  int block_dim;
  int64_t nnzb;
  double density;
  double utilization;
  double average;
} spmm_block_metrics_t;

int spmm_block_metrics(int n, const int* rowptr, const int* colind, int blockDim,
                       spmm_block_metrics_t* out);

/* nnz count of every bs x bs block: heatmap[nb * nb], row-major. */
int spmm_block_heatmap(int n, const int* rowptr, const int* colind, int blockDim, int* heatmap);

/* "nb\n" then nb lines of "c c c ... \n" (utility.cc:90-100 format). */
int spmm_dump_heatmap(const char* filename, int nb, const int* heatmap);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_REORDER_H */
