// multi.cpp — single-process multi-GPU row-partitioned CSR SpMM over RCCL
// (include/spmm_multi.h).
//
// Per call and chunk c: every device p computes its chunk-c rows with the
// 1-GPU merge-path kernel straight into their rows of its own m x n C on its
// compute stream, records an event, and its collective stream waits on that
// event and runs the exchange of chunk c: one ncclGroup in which every device
// ncclSends its chunk-c rows to each peer and ncclRecvs each peer's chunk-c
// rows into the same rows of its C (an all-gather of exact, uneven shards;
// xGMI is point-to-point, so every peer pair has its own link and all of them
// carry data at once). Chunk c+1's kernel is queued on the compute stream
// right away and overlaps chunk c's exchange. At the end each compute stream
// waits for its collective stream, so a caller that synchronises the compute
// stream sees all of C.
//
// RCCL is resolved at run time (dlopen of librccl.so.1 on the first
// spmm_multi_create): the single-GPU entry points of libspmm_hip.so never
// need it, so the library loads on a system without RCCL, and only
// spmm_multi_create reports SPMM_STATUS_NOT_INITIALIZED there. The header is
// included for the types only.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "context.hpp"
#include "spmm_multi.h"

struct spmm_multi {
  int ngpu = 0;
  std::vector<int> dev;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> compute, coll;
  std::vector<spmm_handle_t> handle;
  std::vector<std::vector<hipEvent_t>> chunk_done;  // [p][c]: chunk c's kernel finished
  std::vector<hipEvent_t> t0, t_comp, t_end;         // timing, per part
  std::vector<hipEvent_t> coll_done;                 // [p]: last all-gather finished
  std::vector<hipEvent_t> user_in;                   // [p]: caller's stream reached the call
  std::vector<hipStream_t> user;                     // [p]: caller streams (spmm_multi_set_user_streams)
  bool user_set = false;                             // `user` applies to the next call (NULL = stream 0)
  bool timing = false;
};

namespace {

struct DeviceGuard {
  int saved = 0;
  DeviceGuard() { (void)hipGetDevice(&saved); }
  ~DeviceGuard() { (void)hipSetDevice(saved); }
};

spmm_status_t from_nccl(ncclResult_t r) {
  return r == ncclSuccess ? SPMM_STATUS_SUCCESS : SPMM_STATUS_EXECUTION_FAILED;
}

// The RCCL entry points this file uses, resolved once from librccl.
struct Rccl {
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) return;
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
    r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv;
  });
  return r;
}

#define SPMM_TRY_HIP(x)                                 \
  do {                                                  \
    hipError_t e_ = (x);                                \
    if (e_ != hipSuccess) return spmm::from_hip(e_);    \
  } while (0)

void release(spmm_multi* c) {
  for (int p = 0; p < c->ngpu; ++p) {
    if (p < (int)c->dev.size()) (void)hipSetDevice(c->dev[p]);
    if (p < (int)c->compute.size() && c->compute[p]) (void)hipStreamSynchronize(c->compute[p]);
    if (p < (int)c->coll.size() && c->coll[p]) (void)hipStreamSynchronize(c->coll[p]);
    if (p < (int)c->comm.size() && c->comm[p]) (void)rccl().comm_destroy(c->comm[p]);
    if (p < (int)c->handle.size() && c->handle[p]) (void)spmm_destroy(c->handle[p]);
    if (p < (int)c->chunk_done.size())
      for (auto e : c->chunk_done[p]) (void)hipEventDestroy(e);
    for (auto* v : {&c->t0, &c->t_comp, &c->t_end, &c->coll_done, &c->user_in})
      if (p < (int)v->size() && (*v)[p]) (void)hipEventDestroy((*v)[p]);
    if (p < (int)c->compute.size() && c->compute[p]) (void)hipStreamDestroy(c->compute[p]);
    if (p < (int)c->coll.size() && c->coll[p]) (void)hipStreamDestroy(c->coll[p]);
  }
  delete c;
}

}  // namespace

extern "C" {

spmm_status_t spmm_multi_create(spmm_multi_t* out, int ngpu, const int* devices) {
  if (!out) return SPMM_STATUS_INVALID_VALUE;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return SPMM_STATUS_NOT_INITIALIZED;
  if (ngpu < 1 || ngpu > ndev) return SPMM_STATUS_INVALID_VALUE;
  if (!rccl().ok) return SPMM_STATUS_NOT_INITIALIZED;  // no usable librccl on this system
  std::vector<int> dev(ngpu);
  for (int p = 0; p < ngpu; ++p) {
    dev[p] = devices ? devices[p] : p;
    if (dev[p] < 0 || dev[p] >= ndev) return SPMM_STATUS_INVALID_VALUE;
    for (int q = 0; q < p; ++q)
      if (dev[q] == dev[p]) return SPMM_STATUS_INVALID_VALUE;  // one rank per GPU
  }
  DeviceGuard guard;
  spmm_multi* c = new (std::nothrow) spmm_multi();
  if (!c) return SPMM_STATUS_ALLOC_FAILED;
  c->ngpu = ngpu;
  c->dev = dev;
  c->comm.assign(ngpu, nullptr);
  c->compute.assign(ngpu, nullptr);
  c->coll.assign(ngpu, nullptr);
  c->handle.assign(ngpu, nullptr);
  c->chunk_done.assign(ngpu, {});
  c->t0.assign(ngpu, nullptr);
  c->t_comp.assign(ngpu, nullptr);
  c->t_end.assign(ngpu, nullptr);
  c->coll_done.assign(ngpu, nullptr);
  c->user_in.assign(ngpu, nullptr);
  c->user.assign(ngpu, nullptr);
  spmm_status_t st = SPMM_STATUS_SUCCESS;
  for (int p = 0; p < ngpu && st == SPMM_STATUS_SUCCESS; ++p) {
    hipError_t e = hipSetDevice(dev[p]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->compute[p], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->coll[p], hipStreamNonBlocking);
    for (auto* v : {&c->t0, &c->t_comp, &c->t_end})
      if (e == hipSuccess) e = hipEventCreate(&(*v)[p]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->coll_done[p], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->user_in[p], hipEventDisableTiming);
    if (e != hipSuccess) {
      st = spmm::from_hip(e);
      break;
    }
    st = spmm_create(&c->handle[p]);
    if (st == SPMM_STATUS_SUCCESS) st = spmm_set_stream(c->handle[p], c->compute[p]);
  }
  if (st == SPMM_STATUS_SUCCESS)
    st = from_nccl(rccl().comm_init_all(c->comm.data(), ngpu, dev.data()));
  if (st != SPMM_STATUS_SUCCESS) {
    release(c);
    return st;
  }
  *out = c;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_multi_destroy(spmm_multi_t c) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  DeviceGuard guard;
  release(c);
  return SPMM_STATUS_SUCCESS;
}

int spmm_multi_size(spmm_multi_t c) { return c ? c->ngpu : 0; }

// A NULL entry is the device's legacy null stream (torch's default stream
// reports cuda_stream == 0): the compute and collective streams are
// non-blocking, so nothing would order them against it otherwise. The set
// applies to the next spmm_csr_f32_multi call only, which then forgets it: a
// caller that later destroys one of its streams leaves no dangling handle here.
spmm_status_t spmm_multi_set_user_streams(spmm_multi_t c, void* const* streams) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  c->user_set = streams != nullptr;
  for (int p = 0; p < c->ngpu; ++p)
    c->user[p] = streams ? reinterpret_cast<hipStream_t>(streams[p]) : nullptr;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_multi_get_stream(spmm_multi_t c, int part, void** stream) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  if (!stream || part < 0 || part >= c->ngpu) return SPMM_STATUS_INVALID_VALUE;
  *stream = reinterpret_cast<void*>(c->compute[part]);
  return SPMM_STATUS_SUCCESS;
}

int spmm_multi_slot_rows(int ngpu, const int* bounds, int chunks) {
  if (ngpu < 1 || !bounds || chunks < 1) return 0;
  int mr = 0;
  for (int p = 0; p < ngpu; ++p) mr = std::max(mr, bounds[p + 1] - bounds[p]);
  return std::max(1, (mr + chunks - 1) / chunks);
}

spmm_status_t spmm_csr_f32_multi(spmm_multi_t c, int m, int n, int k, const int* bounds,
                                 const int* const* rowPtr, const int* const* colInd,
                                 const float* const* val, const int* partNnz,
                                 const float* const* B, int ldb, float* const* C, int ldc,
                                 int chunks) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  const int P = c->ngpu;
  if (m < 0 || n < 0 || k < 0 || chunks < 1 || !bounds || !partNnz) return SPMM_STATUS_INVALID_VALUE;
  if (bounds[0] != 0 || bounds[P] != m) return SPMM_STATUS_INVALID_VALUE;
  for (int p = 0; p < P; ++p)
    if (bounds[p + 1] < bounds[p] || partNnz[p] < 0) return SPMM_STATUS_INVALID_VALUE;
  if (m == 0 || n == 0) return SPMM_STATUS_SUCCESS;
  if (!rowPtr || !colInd || !val || !B || !C || ldb < n || ldc < n) return SPMM_STATUS_INVALID_VALUE;
  // the exchange moves spans of whole rows: padding columns would overwrite the peers'
  if (P > 1 && ldc != n) return SPMM_STATUS_NOT_SUPPORTED;
  for (int p = 0; p < P; ++p)
    if (!rowPtr[p] || !C[p] || (k > 0 && !B[p]) || (partNnz[p] > 0 && (!colInd[p] || !val[p])))
      return SPMM_STATUS_INVALID_VALUE;
  const int cr = spmm_multi_slot_rows(P, bounds, chunks);  // rows per chunk
  // part q's chunk ch: local rows [lo, hi), global rows bounds[q] + [lo, hi)
  auto chunk = [&](int q, int ch, int& lo, int& hi) {
    const int rows = bounds[q + 1] - bounds[q];
    lo = std::min(ch * cr, rows);
    hi = std::min(lo + cr, rows);
  };
  // rows r0..r1 of the packed row-major C (ldc == n when P > 1) as one span
  auto span = [&](int r0, int r1) { return (size_t)(r1 - r0) * n; };
  DeviceGuard guard;
  for (int p = 0; p < P; ++p) {
    auto& ev = c->chunk_done[p];
    SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
    while ((int)ev.size() < chunks) {
      hipEvent_t e;
      SPMM_TRY_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ev.push_back(e);
    }
  }
  // inputs produced on the caller's streams are complete before any kernel reads them
  const bool ordered = c->user_set;
  c->user_set = false;  // consumed by this call
  for (int p = 0; p < P && ordered; ++p) {
    SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
    SPMM_TRY_HIP(hipEventRecord(c->user_in[p], c->user[p]));
    SPMM_TRY_HIP(hipStreamWaitEvent(c->compute[p], c->user_in[p], 0));
  }
  for (int ch = 0; ch < chunks; ++ch) {
    for (int p = 0; p < P; ++p) {
      SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
      if (ch == 0 && c->timing) SPMM_TRY_HIP(hipEventRecord(c->t0[p], c->compute[p]));
      const int rows = bounds[p + 1] - bounds[p];
      int r0, r1;
      chunk(p, ch, r0, r1);
      if (r1 > r0) {
        // nnz hint: the part's average share (grid sizing only)
        const int nnz = (int)((long long)partNnz[p] * (r1 - r0) / std::max(rows, 1));
        spmm_status_t st = spmm_csrmm_ex_f32(
            c->handle[p], r1 - r0, n, k, nnz, 1.f, rowPtr[p] + r0, colInd[p], val[p],
            SPMM_INDEX_BASE_ZERO, B[p], ldb, SPMM_ORDER_ROW, 0.f,
            C[p] + (size_t)(bounds[p] + r0) * ldc, ldc, SPMM_ORDER_ROW);
        if (st != SPMM_STATUS_SUCCESS) return st;
      }
      if (ch == chunks - 1 && c->timing) SPMM_TRY_HIP(hipEventRecord(c->t_comp[p], c->compute[p]));
      SPMM_TRY_HIP(hipEventRecord(c->chunk_done[p][ch], c->compute[p]));
      SPMM_TRY_HIP(hipStreamWaitEvent(c->coll[p], c->chunk_done[p][ch], 0));
    }
    if (P == 1) continue;  // one part: nothing to exchange
    // exchange of chunk ch: every (p, q) pair once in each direction, one group
    const Rccl& R = rccl();
    spmm_status_t st = from_nccl(R.group_start());
    for (int p = 0; p < P && st == SPMM_STATUS_SUCCESS; ++p) {
      int m0, m1;
      chunk(p, ch, m0, m1);
      for (int q = 0; q < P && st == SPMM_STATUS_SUCCESS; ++q) {
        if (q == p) continue;
        if (m1 > m0)
          st = from_nccl(R.send(C[p] + (size_t)(bounds[p] + m0) * ldc, span(m0, m1), ncclFloat, q,
                                c->comm[p], c->coll[p]));
        int q0, q1;
        chunk(q, ch, q0, q1);
        if (st == SPMM_STATUS_SUCCESS && q1 > q0)
          st = from_nccl(R.recv(C[p] + (size_t)(bounds[q] + q0) * ldc, span(q0, q1), ncclFloat, q,
                                c->comm[p], c->coll[p]));
      }
    }
    const spmm_status_t st2 = from_nccl(R.group_end());
    if (st != SPMM_STATUS_SUCCESS) return st;
    if (st2 != SPMM_STATUS_SUCCESS) return st2;
  }
  for (int p = 0; p < P; ++p) {
    SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
    SPMM_TRY_HIP(hipEventRecord(c->coll_done[p], c->coll[p]));
    SPMM_TRY_HIP(hipStreamWaitEvent(c->compute[p], c->coll_done[p], 0));
    if (c->timing) SPMM_TRY_HIP(hipEventRecord(c->t_end[p], c->compute[p]));
    // later work on the caller's stream sees all of C
    if (ordered) SPMM_TRY_HIP(hipStreamWaitEvent(c->user[p], c->coll_done[p], 0));
  }
  for (int p = 0; p < P; ++p) c->user[p] = nullptr;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_multi_synchronize(spmm_multi_t c) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  DeviceGuard guard;
  for (int p = 0; p < c->ngpu; ++p) {
    SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
    SPMM_TRY_HIP(hipStreamSynchronize(c->compute[p]));
    SPMM_TRY_HIP(hipStreamSynchronize(c->coll[p]));
  }
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_multi_set_timing(spmm_multi_t c, int enable) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  c->timing = enable != 0;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_multi_get_times(spmm_multi_t c, float* compute_ms, float* total_ms) {
  if (!c) return SPMM_STATUS_NOT_INITIALIZED;
  if (!compute_ms || !total_ms) return SPMM_STATUS_INVALID_VALUE;
  if (!c->timing) return SPMM_STATUS_INVALID_VALUE;
  DeviceGuard guard;
  for (int p = 0; p < c->ngpu; ++p) {
    SPMM_TRY_HIP(hipSetDevice(c->dev[p]));
    SPMM_TRY_HIP(hipEventSynchronize(c->t_end[p]));
    SPMM_TRY_HIP(hipEventElapsedTime(&compute_ms[p], c->t0[p], c->t_comp[p]));
    SPMM_TRY_HIP(hipEventElapsedTime(&total_ms[p], c->t0[p], c->t_end[p]));
  }
  return SPMM_STATUS_SUCCESS;
}

}  // extern "C"
