// host_io.cpp — graph/matrix files (include/spmm_host.h): the reference's
// text formats, parsed and written in parallel, plus a checksummed binary
// sidecar cache.
//
//   dumpCSRToFile / loadCSRFromFile   load_data.cc:125-165  "<n+1>\n r0 r1 ... \n" /
//                                                           "<nnz>\n c0 c1 ... \n"
//   loadGraphFromFile                 load_data.cc:167-184  "n nnz\n" then nnz "src dst"
//                                                           pairs; lists sorted, duplicates kept
//
// Text is read whole and tokenised by worker threads (each chunk starts at a
// token boundary; counts, prefix sum, parse), so products-scale files load
// in a fraction of a second instead of the several seconds a stream parse
// takes. The results are exactly what the reference's iostream loops give on
// well-formed files; malformed input returns -1 instead of garbage.
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host_util.hpp"
#include "spmm_host.h"

using spmm_host::num_threads;
using spmm_host::parallel_for;

namespace {

bool read_file(const std::string& path, std::vector<char>& buf) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(sz > 0 ? (size_t)sz : 0);
  const size_t got = sz > 0 ? std::fread(buf.data(), 1, (size_t)sz, f) : 0;
  std::fclose(f);
  return got == buf.size();
}

inline bool is_space(char c) { return (unsigned char)c <= ' '; }

// Parses every whitespace-separated integer of buf[begin, end) into out
// (which must have room for them); returns the count or -1 on a bad token.
// Parallel: chunks start after a whitespace byte.
template <typename T>
int64_t parse_ints(const char* buf, size_t begin, size_t end, T* out, int64_t expect) {
  const int nt = std::max(1, std::min<int>(num_threads(), (int)((end - begin) >> 20) + 1));
  std::vector<size_t> cut(nt + 1);
  cut[0] = begin;
  cut[nt] = end;
  for (int t = 1; t < nt; ++t) {
    size_t c = begin + (end - begin) * t / nt;
    while (c < end && !is_space(buf[c])) ++c;  // move to a token boundary
    cut[t] = std::max(c, cut[t - 1]);
  }
  std::vector<int64_t> cnt(nt + 1, 0);
  std::atomic<bool> bad{false};
  auto count = [&](int t) {
    int64_t c = 0;
    bool in = false;
    for (size_t i = cut[t]; i < cut[t + 1]; ++i) {
      const bool sp = is_space(buf[i]);
      if (!sp && !in) ++c;
      in = !sp;
    }
    cnt[t + 1] = c;
  };
  auto parse = [&](int t, int64_t pos) {
    size_t i = cut[t];
    const size_t e = cut[t + 1];
    while (i < e) {
      while (i < e && is_space(buf[i])) ++i;
      if (i >= e) break;
      size_t j = i;
      while (j < e && !is_space(buf[j])) ++j;
      T v{};
      const auto r = std::from_chars(buf + i, buf + j, v);
      if (r.ec != std::errc() || r.ptr != buf + j) {
        bad = true;
        return;
      }
      if (pos < expect) out[pos] = v;
      ++pos;
      i = j;
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(count, t);
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
  if (cnt[nt] < expect) return -1;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(parse, t, cnt[t]);
    for (auto& x : th) x.join();
  }
  return bad ? -1 : cnt[nt];
}

// Parses the integer token starting at or after `from`; `after` is set just
// past it.
bool next_token(const std::vector<char>& buf, size_t from, long long& v, size_t& after) {
  size_t i = from;
  while (i < buf.size() && is_space(buf[i])) ++i;
  size_t j = i;
  while (j < buf.size() && !is_space(buf[j])) ++j;
  const auto r = std::from_chars(buf.data() + i, buf.data() + j, v);
  if (i == j || r.ec != std::errc() || r.ptr != buf.data() + j) return false;
  after = j;
  return true;
}

// Writes "v v v ... \n" (each value followed by one space) like the
// reference's `s << x << " "` loop, formatted by worker threads.
template <typename T>
bool write_ints(FILE* f, const T* v, int64_t n) {
  const int64_t per = 1 << 20;
  const int64_t chunks = (n + per - 1) / per;
  std::vector<std::string> parts((size_t)std::max<int64_t>(chunks, 0));
  parallel_for(chunks, [&](int64_t lo, int64_t hi) {
    char tmp[24];
    for (int64_t c = lo; c < hi; ++c) {
      std::string& s = parts[c];
      const int64_t a = c * per, b = std::min(n, a + per);
      s.reserve((size_t)(b - a) * 9);
      for (int64_t i = a; i < b; ++i) {
        const auto r = std::to_chars(tmp, tmp + sizeof tmp, v[i]);
        s.append(tmp, r.ptr);
        s.push_back(' ');
      }
    }
  });
  for (const auto& s : parts)
    if (std::fwrite(s.data(), 1, s.size(), f) != s.size()) return false;
  return true;
}

// ---------------------------------------------------------------- checksum
// 64-bit, order-sensitive, computed over 1 MiB chunks in parallel and folded
// in chunk order (a corruption detector, not a cryptographic hash).
inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

uint64_t checksum(const void* data, size_t bytes, uint64_t seed) {
  const unsigned char* p = static_cast<const unsigned char*>(data);
  const size_t per = 1 << 20;
  const size_t chunks = (bytes + per - 1) / per;
  std::vector<uint64_t> hs(chunks);
  parallel_for((int64_t)chunks, [&](int64_t lo, int64_t hi) {
    for (int64_t c = lo; c < hi; ++c) {
      const size_t a = (size_t)c * per, b = std::min(bytes, a + per);
      uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)c;
      size_t i = a;
      for (; i + 8 <= b; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
      }
      uint64_t tail = 0;
      std::memcpy(&tail, p + i, b - i);
      hs[c] = mix64(h ^ tail ^ (uint64_t)(b - a));
    }
  });
  uint64_t h = mix64(seed ^ bytes);
  for (uint64_t x : hs) h = mix64(h ^ x) + 0x632be59bd9b4e019ull;
  return h;
}

struct BinHeader {
  char magic[8];  // "SPMMCSR1"
  uint32_t version;
  uint32_t flags;  // bit 0: float values follow colind
  int64_t n;
  int64_t nnz;
  uint64_t sum_rowptr, sum_colind, sum_val;
};
constexpr char kMagic[8] = {'S', 'P', 'M', 'M', 'C', 'S', 'R', '1'};

int64_t mtime_ns(const std::string& path) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return -1;
  return (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
}

}  // namespace

extern "C" {

int spmm_host_dump_csr(const char* prefix, int n, int64_t nnz, const int* rowptr,
                       const int* colind) {
  if (!prefix || n < 0 || !rowptr || nnz < 0 || (nnz > 0 && !colind)) return -1;
  const std::string p(prefix);
  FILE* f1 = std::fopen((p + "_indptr.txt").c_str(), "wb");
  FILE* f2 = std::fopen((p + "_indices.txt").c_str(), "wb");
  bool ok = f1 && f2;
  if (ok) {
    ok = std::fprintf(f1, "%d\n", n + 1) > 0 && write_ints(f1, rowptr, (int64_t)n + 1) &&
         std::fputc('\n', f1) != EOF;
    ok = ok && std::fprintf(f2, "%lld\n", (long long)nnz) > 0 && write_ints(f2, colind, nnz) &&
         std::fputc('\n', f2) != EOF;
  }
  if (f1 && std::fclose(f1) != 0) ok = false;
  if (f2 && std::fclose(f2) != 0) ok = false;
  return ok ? 0 : -1;
}

int spmm_host_load_csr(const char* prefix, int** rowptr, int** colind, int* n, int64_t* nnz) {
  if (!prefix || !rowptr || !colind || !n || !nnz) return -1;
  const std::string p(prefix);
  std::vector<char> b1, b2;
  if (!read_file(p + "_indptr.txt", b1) || !read_file(p + "_indices.txt", b2)) return -1;
  long long np1 = 0, z = 0;
  size_t a1 = 0, a2 = 0;
  if (!next_token(b1, 0, np1, a1) || np1 < 1 || np1 - 1 > INT32_MAX) return -1;
  if (!next_token(b2, 0, z, a2) || z < 0) return -1;
  int* rp = static_cast<int*>(std::malloc(sizeof(int) * (size_t)np1));
  int* ci = static_cast<int*>(std::malloc(sizeof(int) * (size_t)std::max(1LL, z)));
  if (!rp || !ci || parse_ints(b1.data(), a1, b1.size(), rp, np1) < 0 ||
      parse_ints(b2.data(), a2, b2.size(), ci, z) < 0) {
    std::free(rp);
    std::free(ci);
    return -1;
  }
  *rowptr = rp;
  *colind = ci;
  *n = (int)(np1 - 1);
  *nnz = z;
  return 0;
}

int spmm_host_load_graph(const char* filename, int** rowptr, int** colind, int* n_out,
                         int64_t* nnz_out) {
  if (!filename || !rowptr || !colind || !n_out || !nnz_out) return -1;
  std::vector<char> buf;
  if (!read_file(filename, buf)) return -1;
  long long hdr[2];
  size_t a = 0, pos = 0;
  if (!next_token(buf, 0, hdr[0], a) || !next_token(buf, a, hdr[1], pos)) return -1;
  const long long n = hdr[0], nnz = hdr[1];
  if (n < 0 || n > INT32_MAX || nnz < 0 || nnz > INT32_MAX) return -1;
  std::vector<int> ed((size_t)2 * nnz);
  if (parse_ints(buf.data(), pos, buf.size(), ed.data(), 2 * nnz) < 0) return -1;
  buf.clear();
  buf.shrink_to_fit();
  // Counting sort by source (stable: input order inside a row), then each
  // row sorted — the reference's push_back + std::sort per list.
  std::vector<int> rp((size_t)n + 1, 0);
  for (long long e = 0; e < nnz; ++e) {
    const int x = ed[2 * e];
    if (x < 0 || x >= n) return -1;
    ++rp[x + 1];
  }
  for (long long i = 0; i < n; ++i) rp[i + 1] += rp[i];
  std::vector<int> ci((size_t)std::max(1LL, nnz));
  {
    std::vector<int> fill(rp.begin(), rp.end() - 1);
    for (long long e = 0; e < nnz; ++e) ci[fill[ed[2 * e]]++] = ed[2 * e + 1];
  }
  parallel_for(n, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) std::sort(ci.begin() + rp[i], ci.begin() + rp[i + 1]);
  });
  int* rpo = static_cast<int*>(std::malloc(sizeof(int) * ((size_t)n + 1)));
  int* cio = static_cast<int*>(std::malloc(sizeof(int) * (size_t)std::max(1LL, nnz)));
  if (!rpo || !cio) {
    std::free(rpo);
    std::free(cio);
    return -1;
  }
  std::memcpy(rpo, rp.data(), sizeof(int) * ((size_t)n + 1));
  if (nnz) std::memcpy(cio, ci.data(), sizeof(int) * (size_t)nnz);
  *rowptr = rpo;
  *colind = cio;
  *n_out = (int)n;
  *nnz_out = nnz;
  return 0;
}

int spmm_host_save_csr_bin(const char* path, int n, int64_t nnz, const int* rowptr,
                           const int* colind, const float* val) {
  if (!path || n < 0 || nnz < 0 || !rowptr || (nnz > 0 && !colind)) return -1;
  BinHeader h{};
  std::memcpy(h.magic, kMagic, 8);
  h.version = 1;
  h.flags = val ? 1u : 0u;
  h.n = n;
  h.nnz = nnz;
  h.sum_rowptr = checksum(rowptr, sizeof(int) * ((size_t)n + 1), 1);
  h.sum_colind = checksum(colind, sizeof(int) * (size_t)nnz, 2);
  h.sum_val = val ? checksum(val, sizeof(float) * (size_t)nnz, 3) : 0;
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return -1;
  bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
            std::fwrite(rowptr, sizeof(int), (size_t)n + 1, f) == (size_t)n + 1 &&
            (nnz == 0 || std::fwrite(colind, sizeof(int), (size_t)nnz, f) == (size_t)nnz) &&
            (!val || nnz == 0 || std::fwrite(val, sizeof(float), (size_t)nnz, f) == (size_t)nnz);
  if (std::fclose(f) != 0) ok = false;
  // Written under a temporary name and renamed: a reader never sees a
  // half-written cache.
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    return -1;
  }
  return 0;
}

int spmm_host_load_csr_bin(const char* path, int** rowptr, int** colind, float** val, int* n,
                           int64_t* nnz) {
  if (!path || !rowptr || !colind || !n || !nnz) return -1;
  FILE* f = std::fopen(path, "rb");
  if (!f) return -1;
  BinHeader h{};
  if (std::fread(&h, sizeof h, 1, f) != 1 || std::memcmp(h.magic, kMagic, 8) != 0 ||
      h.version != 1 || h.n < 0 || h.n > INT32_MAX || h.nnz < 0) {
    std::fclose(f);
    return -1;
  }
  int* rp = static_cast<int*>(std::malloc(sizeof(int) * ((size_t)h.n + 1)));
  int* ci = static_cast<int*>(std::malloc(sizeof(int) * (size_t)std::max<int64_t>(1, h.nnz)));
  float* v = (h.flags & 1) ? static_cast<float*>(std::malloc(
                                 sizeof(float) * (size_t)std::max<int64_t>(1, h.nnz)))
                           : nullptr;
  bool ok = rp && ci && (!(h.flags & 1) || v);
  ok = ok && std::fread(rp, sizeof(int), (size_t)h.n + 1, f) == (size_t)h.n + 1;
  ok = ok && (h.nnz == 0 || std::fread(ci, sizeof(int), (size_t)h.nnz, f) == (size_t)h.nnz);
  ok = ok && (!v || h.nnz == 0 || std::fread(v, sizeof(float), (size_t)h.nnz, f) == (size_t)h.nnz);
  std::fclose(f);
  int rc = ok ? 0 : -1;
  if (ok && (checksum(rp, sizeof(int) * ((size_t)h.n + 1), 1) != h.sum_rowptr ||
             checksum(ci, sizeof(int) * (size_t)h.nnz, 2) != h.sum_colind ||
             (v && checksum(v, sizeof(float) * (size_t)h.nnz, 3) != h.sum_val)))
    rc = -2;
  if (rc != 0 || (!val && v)) {
    if (rc != 0) {
      std::free(rp);
      std::free(ci);
    }
    std::free(v);
    v = nullptr;
    if (rc != 0) return rc;
  }
  *rowptr = rp;
  *colind = ci;
  if (val) *val = v;
  *n = (int)h.n;
  *nnz = h.nnz;
  return 0;
}

int spmm_host_load_csr_cached(const char* prefix, int** rowptr, int** colind, int* n,
                              int64_t* nnz) {
  if (!prefix) return -1;
  const std::string p(prefix), bin = p + ".csrbin";
  const int64_t t_bin = mtime_ns(bin);
  const int64_t t_txt = std::max(mtime_ns(p + "_indptr.txt"), mtime_ns(p + "_indices.txt"));
  if (t_bin >= 0 && t_bin >= t_txt &&
      spmm_host_load_csr_bin(bin.c_str(), rowptr, colind, nullptr, n, nnz) == 0)
    return 0;  // fresh, intact cache
  const int rc = spmm_host_load_csr(prefix, rowptr, colind, n, nnz);
  if (rc == 0) spmm_host_save_csr_bin(bin.c_str(), *n, *nnz, *rowptr, *colind, nullptr);
  return rc;
}

}  // extern "C"
