// host_util.hpp — shared host-side helpers of libspmm_hip.so (threads only).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace spmm_host {

// Worker count: OMP_NUM_THREADS if set, else the hardware threads, capped at 32.
inline int num_threads() {
  unsigned t = std::thread::hardware_concurrency();
  if (const char* e = std::getenv("OMP_NUM_THREADS")) t = (unsigned)std::max(1, std::atoi(e));
  return (int)std::max(1u, std::min(t, 32u));
}

// Runs f(lo, hi) over [0, n) in contiguous chunks on worker threads.
template <typename F>
void parallel_for(int64_t n, F f) {
  const int nt = (int)std::min<int64_t>(num_threads(), std::max<int64_t>(1, n / 4096));
  if (nt <= 1) {
    f((int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    th.emplace_back([=] { f(lo, hi); });
  }
  for (auto& x : th) x.join();
}

}  // namespace spmm_host
