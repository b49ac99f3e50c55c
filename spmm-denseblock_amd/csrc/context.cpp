// context.cpp — handle lifecycle, workspace and kernel-timing ring.
#include "context.hpp"

#include <new>

namespace spmm {

static spmm_status_t grow_buffer(spmm_context* ctx, void*& buf, size_t& cap, size_t bytes) {
  if (bytes <= cap) return SPMM_STATUS_SUCCESS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (bytes <= cap) return SPMM_STATUS_SUCCESS;
  // The old buffer may still be in use by queued work on this stream.
  if (buf) {
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return from_hip(e);
    (void)hipFree(buf);
    buf = nullptr;
    cap = 0;
  }
  size_t want = bytes + bytes / 4;  // grow with slack
  hipError_t e = hipMalloc(&buf, want);
  if (e != hipSuccess) {
    buf = nullptr;
    return from_hip(e);
  }
  cap = want;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t ensure_workspace(spmm_context* ctx, size_t bytes) {
  return grow_buffer(ctx, ctx->ws, ctx->ws_bytes, bytes);
}

spmm_status_t ensure_scratch(spmm_context* ctx, size_t bytes) {
  return grow_buffer(ctx, ctx->scratch, ctx->scratch_bytes, bytes);
}

spmm_status_t ensure_group_pending(spmm_context* ctx, size_t bytes) {
  return grow_buffer(ctx, ctx->grp_pend, ctx->grp_pend_bytes, bytes);
}

spmm_status_t ensure_order_buffer(spmm_context* ctx, size_t n) {
  if (n <= ctx->order_cap) return SPMM_STATUS_SUCCESS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n <= ctx->order_cap) return SPMM_STATUS_SUCCESS;
  if (ctx->order) {
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return from_hip(e);
    (void)hipFree(ctx->order);
    ctx->order = nullptr;
    ctx->order_cap = 0;
  }
  const size_t want = n + n / 4 + 1024;
  hipError_t e = hipMalloc(&ctx->order, want * sizeof(int));
  if (e != hipSuccess) {
    ctx->order = nullptr;
    return from_hip(e);
  }
  ctx->order_cap = want;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t ensure_tickets(spmm_context* ctx, size_t n) {
  if (n <= ctx->tickets_cap) return SPMM_STATUS_SUCCESS;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n <= ctx->tickets_cap) return SPMM_STATUS_SUCCESS;
  if (ctx->tickets) {
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return from_hip(e);
    (void)hipFree(ctx->tickets);
    ctx->tickets = nullptr;
    ctx->tickets_cap = 0;
  }
  const size_t want = n + n / 4 + 1024;
  hipError_t e = hipMalloc(&ctx->tickets, want * sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(ctx->tickets, 0, want * sizeof(int), ctx->stream);
  if (e != hipSuccess) {
    if (ctx->tickets) (void)hipFree(ctx->tickets);
    ctx->tickets = nullptr;
    return from_hip(e);
  }
  ctx->tickets_cap = want;
  return SPMM_STATUS_SUCCESS;
}

int timing_begin(spmm_context* ctx) {
  if (!ctx->timing) return -1;
  const size_t slot = ctx->ev_used;
  if (slot == ctx->ev_start.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return -1;
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      return -1;
    }
    ctx->ev_start.push_back(a);
    ctx->ev_stop.push_back(b);
  }
  (void)hipEventRecord(ctx->ev_start[slot], ctx->stream);
  ctx->ev_used = slot + 1;
  return (int)slot;
}

void timing_end(spmm_context* ctx, int slot) {
  if (slot < 0) return;
  (void)hipEventRecord(ctx->ev_stop[slot], ctx->stream);
}

static spmm_context* make_context() {
  spmm_context* ctx = new (std::nothrow) spmm_context();
  if (!ctx) return nullptr;
  (void)hipGetDevice(&ctx->device);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) ==
          hipSuccess &&
      cus > 0)
    ctx->num_cus = cus;
  return ctx;
}

spmm_context* default_context() {
  // One default handle per device, created on first use.
  static std::mutex mu;
  static spmm_context* ctxs[64] = {nullptr};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!ctxs[dev]) ctxs[dev] = make_context();
  return ctxs[dev];
}

}  // namespace spmm

using namespace spmm;

extern "C" {

int spmm_get_version(void) { return SPMM_HIP_VERSION; }

const char* spmm_get_status_string(spmm_status_t s) {
  switch (s) {
    case SPMM_STATUS_SUCCESS: return "SPMM_STATUS_SUCCESS";
    case SPMM_STATUS_NOT_INITIALIZED: return "SPMM_STATUS_NOT_INITIALIZED";
    case SPMM_STATUS_ALLOC_FAILED: return "SPMM_STATUS_ALLOC_FAILED";
    case SPMM_STATUS_INVALID_VALUE: return "SPMM_STATUS_INVALID_VALUE";
    case SPMM_STATUS_ARCH_MISMATCH: return "SPMM_STATUS_ARCH_MISMATCH";
    case SPMM_STATUS_MAPPING_ERROR: return "SPMM_STATUS_MAPPING_ERROR";
    case SPMM_STATUS_EXECUTION_FAILED: return "SPMM_STATUS_EXECUTION_FAILED";
    case SPMM_STATUS_INTERNAL_ERROR: return "SPMM_STATUS_INTERNAL_ERROR";
    case SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED: return "SPMM_STATUS_MATRIX_TYPE_NOT_SUPPORTED";
    case SPMM_STATUS_ZERO_PIVOT: return "SPMM_STATUS_ZERO_PIVOT";
    case SPMM_STATUS_NOT_SUPPORTED: return "SPMM_STATUS_NOT_SUPPORTED";
  }
  return "SPMM_STATUS_UNKNOWN";
}

spmm_status_t spmm_create(spmm_handle_t* handle) {
  if (!handle) return SPMM_STATUS_INVALID_VALUE;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    *handle = nullptr;
    return SPMM_STATUS_NOT_INITIALIZED;
  }
  *handle = make_context();
  return *handle ? SPMM_STATUS_SUCCESS : SPMM_STATUS_ALLOC_FAILED;
}

spmm_status_t spmm_destroy(spmm_handle_t h) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (h->grp_cols) (void)hipFreeAsync(h->grp_cols, h->stream);
  if (h->ws || h->scratch || h->order || h->tickets || h->grp_pend || h->grp_cols)
    (void)hipStreamSynchronize(h->stream);
  if (h->ws) (void)hipFree(h->ws);
  if (h->grp_pend) (void)hipFree(h->grp_pend);
  if (h->tickets) (void)hipFree(h->tickets);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->order) (void)hipFree(h->order);
  for (auto e : h->ev_start) (void)hipEventDestroy(e);
  for (auto e : h->ev_stop) (void)hipEventDestroy(e);
  delete h;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_stream(spmm_handle_t h, void* stream) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  h->stream = reinterpret_cast<hipStream_t>(stream);
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_get_stream(spmm_handle_t h, void** stream) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (!stream) return SPMM_STATUS_INVALID_VALUE;
  *stream = reinterpret_cast<void*>(h->stream);
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_create_mat_descr(spmm_mat_descr_t* d) {
  if (!d) return SPMM_STATUS_INVALID_VALUE;
  *d = new (std::nothrow) spmm_mat_descr();
  return *d ? SPMM_STATUS_SUCCESS : SPMM_STATUS_ALLOC_FAILED;
}

spmm_status_t spmm_destroy_mat_descr(spmm_mat_descr_t d) {
  delete d;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_mat_type(spmm_mat_descr_t d, spmm_matrix_type_t t) {
  if (!d || t != SPMM_MATRIX_TYPE_GENERAL) return SPMM_STATUS_INVALID_VALUE;
  d->type = t;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_mat_index_base(spmm_mat_descr_t d, spmm_index_base_t b) {
  if (!d || (b != SPMM_INDEX_BASE_ZERO && b != SPMM_INDEX_BASE_ONE))
    return SPMM_STATUS_INVALID_VALUE;
  d->base = b;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_kernel_timing(spmm_handle_t h, int enable) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  h->timing = enable != 0;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_get_kernel_times(spmm_handle_t h, float* ms, int max_count, int* count) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (!count || (max_count > 0 && !ms)) return SPMM_STATUS_INVALID_VALUE;
  int c = 0;
  for (size_t s = 0; s < h->ev_used && c < max_count; ++s) {
    hipError_t e = hipEventSynchronize(h->ev_stop[s]);
    if (e != hipSuccess) return from_hip(e);
    float t = 0.f;
    e = hipEventElapsedTime(&t, h->ev_start[s], h->ev_stop[s]);
    if (e != hipSuccess) return from_hip(e);
    ms[c++] = t;
  }
  *count = c;
  h->ev_used = 0;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_csr_waves_per_cu(spmm_handle_t h, int w) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (w < 0 || w > 32) return SPMM_STATUS_INVALID_VALUE;
  h->csr_waves_per_cu = w;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_csr_options(spmm_handle_t h, int flags) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (flags & ~(SPMM_CSR_NT_STREAMS | SPMM_CSR_SEQUENTIAL_ROWS)) return SPMM_STATUS_INVALID_VALUE;
  h->csr_flags = flags;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_hybrid_options(spmm_handle_t h, int flags) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if ((flags & ~(SPMM_HYBRID_FUSED | SPMM_HYBRID_TWO_LAUNCH | SPMM_HYBRID_SPLIT_BF16)) ||
      (flags & SPMM_HYBRID_FUSED && flags & SPMM_HYBRID_TWO_LAUNCH))
    return SPMM_STATUS_INVALID_VALUE;
  h->hybrid_flags = flags;
  return SPMM_STATUS_SUCCESS;
}

spmm_status_t spmm_set_bsr_options(spmm_handle_t h, int flags) {
  if (!h) return SPMM_STATUS_NOT_INITIALIZED;
  if (flags & ~(SPMM_BSR_DENSE_BLOCK_PRODUCT | SPMM_BSR_SMALL_GROUPED)) return SPMM_STATUS_INVALID_VALUE;
  h->bsr_flags = flags;
  return SPMM_STATUS_SUCCESS;
}

int spmm_get_build_options(void) {
#ifdef SPMM_TUNING
  return SPMM_BUILD_TUNING;
#else
  return 0;
#endif
}

}  // extern "C"
