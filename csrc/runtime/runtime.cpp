// Host runtime for flexible_llm_sharding_amd (MI355X).
//
// * pinned host memory (hipHostMalloc / hipHostRegister) for weight slots
//   and activation spill rings — allocated once, no malloc_trim games
//   (reference: utils.py:18-21 clean_memory);
// * a multi-threaded pread/pwrite engine that reads safetensors tensor bytes
//   straight into pinned destinations (reference reads whole files into a
//   Python bytes object and deserializes: utils.py:126-127) and writes
//   activation spill files (reference: np.save, utils.py:171-177);
// * a block gather used to repack weights into the HBM-native layout;
// * a safetensors header index (8-byte length + JSON) with a small JSON
//   scanner specialised for the format.
//
// Built with g++ against libamdhip64 (host code only).
#include "fls.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

extern "C" int fls_rt_version(void) { return 1; }

// ------------------------------------------------------------------ pinned
extern "C" void* fls_pinned_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (bytes == 0) bytes = 1;
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
  if (e != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  return p;
}

extern "C" int fls_pinned_free(void* p) {
  if (!p) return 0;
  return hipHostFree(p) == hipSuccess ? 0 : -1;
}

extern "C" int fls_pinned_register(void* p, uint64_t bytes) {
  return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? 0 : -1;
}

extern "C" int fls_pinned_unregister(void* p) {
  return hipHostUnregister(p) == hipSuccess ? 0 : -1;
}

extern "C" int fls_memcpy_async(void* dst, const void* src, uint64_t bytes, int kind, fls_stream_t s) {
  hipMemcpyKind k = hipMemcpyDefault;
  if (kind == 1) k = hipMemcpyHostToDevice;
  else if (kind == 2) k = hipMemcpyDeviceToHost;
  else if (kind == 3) k = hipMemcpyDeviceToDevice;
  return hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)s) == hipSuccess ? 0 : -1;
}

extern "C" int fls_mem_info(uint64_t* free_b, uint64_t* total_b) {
  size_t f = 0, t = 0;
  if (hipMemGetInfo(&f, &t) != hipSuccess) return -1;
  *free_b = f; *total_b = t;
  return 0;
}

// ------------------------------------------------------------ file engine
namespace {
constexpr uint64_t kChunk = 16ull << 20;   // 16 MiB pread granules

int64_t parallel_io(int fd, uint64_t offset, uint64_t bytes, char* buf, int nthreads, bool write) {
  if (bytes == 0) return 0;
  uint64_t nchunks = (bytes + kChunk - 1) / kChunk;
  int nt = std::max(1, std::min<int>(nthreads, (int)nchunks));
  std::atomic<uint64_t> next{0};
  std::atomic<int64_t> err{0};
  auto work = [&]() {
    for (;;) {
      uint64_t c = next.fetch_add(1);
      if (c >= nchunks || err.load()) return;
      uint64_t lo = c * kChunk, n = std::min<uint64_t>(kChunk, bytes - lo);
      uint64_t done = 0;
      while (done < n) {
        ssize_t r = write ? pwrite(fd, buf + lo + done, n - done, offset + lo + done)
                          : pread(fd, buf + lo + done, n - done, offset + lo + done);
        if (r < 0) { if (errno == EINTR) continue; err.store(-errno); return; }
        if (r == 0) { err.store(-EIO); return; }   // unexpected EOF
        done += (uint64_t)r;
      }
    }
  };
  if (nt == 1) { work(); }
  else {
    std::vector<std::thread> ts;
    for (int i = 0; i < nt; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
  }
  return err.load() ? err.load() : (int64_t)bytes;
}
}  // namespace

extern "C" int64_t fls_pread_into(const char* path, uint64_t offset, uint64_t bytes, void* dst,
                                  int nthreads) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  posix_fadvise(fd, (off_t)offset, (off_t)bytes, POSIX_FADV_SEQUENTIAL);
  int64_t r = parallel_io(fd, offset, bytes, (char*)dst, nthreads, false);
  close(fd);
  return r;
}

extern "C" int64_t fls_pwrite_from(const char* path, uint64_t offset, uint64_t bytes, const void* src,
                                   int nthreads, int truncate) {
  int flags = O_WRONLY | O_CREAT | O_CLOEXEC | (truncate ? O_TRUNC : 0);
  int fd = open(path, flags, 0644);
  if (fd < 0) return -errno;
  int64_t r = parallel_io(fd, offset, bytes, (char*)const_cast<void*>(src), nthreads, true);
  close(fd);
  return r;
}

extern "C" int fls_gather_blocks(void* dst, const void* src, uint64_t block_bytes,
                                 const int64_t* src_block, int64_t n_blocks, int nthreads) {
  char* d = (char*)dst;
  const char* s = (const char*)src;
  int nt = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, n_blocks / 4)));
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (;;) {
      int64_t i = next.fetch_add(64);
      if (i >= n_blocks) return;
      int64_t e = std::min<int64_t>(n_blocks, i + 64);
      for (; i < e; ++i) std::memcpy(d + (uint64_t)i * block_bytes, s + (uint64_t)src_block[i] * block_bytes, block_bytes);
    }
  };
  if (nt == 1) work();
  else {
    std::vector<std::thread> ts;
    for (int i = 0; i < nt; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
  }
  return 0;
}

// ------------------------------------------------------- safetensors index
namespace {
struct StEntry {
  std::string name, dtype;
  std::vector<int64_t> shape;
  uint64_t begin = 0, end = 0;
};
struct StFile {
  std::vector<StEntry> entries;
  uint64_t data_off = 0;
};

struct Scanner {
  const char* p; const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
  std::string str() {
    ws();
    std::string out;
    if (p >= e || *p != '"') { ok = false; return out; }
    ++p;
    while (p < e && *p != '"') {
      if (*p == '\\' && p + 1 < e) {
        ++p;
        switch (*p) {
          case 'n': out += '\n'; break; case 't': out += '\t'; break;
          case 'u': {  // keep escaped code units verbatim (names are ASCII in practice)
            out += "\\u"; break; }
          default: out += *p;
        }
        ++p;
      } else out += *p++;
    }
    if (p >= e) { ok = false; return out; }
    ++p;
    return out;
  }
  int64_t num() {
    ws();
    char* end = nullptr;
    long long v = std::strtoll(p, &end, 10);
    if (end == p) ok = false;
    p = end;
    return (int64_t)v;
  }
  void skip_value() {   // skip any JSON value
    ws();
    if (p >= e) { ok = false; return; }
    if (*p == '"') { str(); return; }
    if (*p == '{' || *p == '[') {
      char open = *p, close = (*p == '{') ? '}' : ']';
      int depth = 0;
      bool in_str = false;
      for (; p < e; ++p) {
        if (in_str) { if (*p == '\\') ++p; else if (*p == '"') in_str = false; continue; }
        if (*p == '"') in_str = true;
        else if (*p == open) ++depth;
        else if (*p == close) { if (--depth == 0) { ++p; return; } }
      }
      ok = false; return;
    }
    while (p < e && *p != ',' && *p != '}' && *p != ']') ++p;
  }
};

bool parse_entry(Scanner& sc, StEntry& en) {
  if (!sc.eat('{')) return false;
  bool first = true;
  while (sc.ok) {
    if (sc.eat('}')) return true;
    if (!first && !sc.eat(',')) return false;
    first = false;
    std::string k = sc.str();
    if (!sc.eat(':')) return false;
    if (k == "dtype") en.dtype = sc.str();
    else if (k == "shape") {
      if (!sc.eat('[')) return false;
      if (!sc.eat(']')) {
        do { en.shape.push_back(sc.num()); } while (sc.eat(','));
        if (!sc.eat(']')) return false;
      }
    } else if (k == "data_offsets") {
      if (!sc.eat('[')) return false;
      en.begin = (uint64_t)sc.num();
      if (!sc.eat(',')) return false;
      en.end = (uint64_t)sc.num();
      if (!sc.eat(']')) return false;
    } else sc.skip_value();
  }
  return false;
}
}  // namespace

extern "C" void* fls_st_open(const char* path) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return nullptr;
  uint64_t n = 0;
  if (pread(fd, &n, 8, 0) != 8 || n > (100ull << 20)) { close(fd); return nullptr; }
  std::string hdr(n, '\0');
  if ((uint64_t)pread(fd, &hdr[0], n, 8) != n) { close(fd); return nullptr; }
  close(fd);
  auto* f = new StFile();
  f->data_off = 8 + n;
  Scanner sc{hdr.data(), hdr.data() + hdr.size()};
  if (!sc.eat('{')) { delete f; return nullptr; }
  bool first = true;
  while (sc.ok) {
    if (sc.eat('}')) break;
    if (!first && !sc.eat(',')) { sc.ok = false; break; }
    first = false;
    std::string key = sc.str();
    if (!sc.eat(':')) { sc.ok = false; break; }
    if (key == "__metadata__") { sc.skip_value(); continue; }
    StEntry en;
    en.name = key;
    if (!parse_entry(sc, en)) { sc.ok = false; break; }
    f->entries.push_back(std::move(en));
  }
  if (!sc.ok) { delete f; return nullptr; }
  return f;
}

extern "C" int fls_st_count(void* h) { return h ? (int)((StFile*)h)->entries.size() : -1; }

extern "C" uint64_t fls_st_data_offset(void* h) { return h ? ((StFile*)h)->data_off : 0; }

extern "C" int fls_st_info(void* h, int i, char* name, int name_cap, char* dtype, int dtype_cap,
                           int64_t* shape, int* ndim, uint64_t* begin, uint64_t* end) {
  auto* f = (StFile*)h;
  if (!f || i < 0 || i >= (int)f->entries.size()) return -1;
  const StEntry& en = f->entries[i];
  if ((int)en.name.size() + 1 > name_cap || (int)en.dtype.size() + 1 > dtype_cap) return -2;
  std::memcpy(name, en.name.c_str(), en.name.size() + 1);
  std::memcpy(dtype, en.dtype.c_str(), en.dtype.size() + 1);
  int nd = (int)en.shape.size();
  if (nd > 8) return -3;
  for (int d = 0; d < nd; ++d) shape[d] = en.shape[d];
  *ndim = nd;
  *begin = f->data_off + en.begin;
  *end = f->data_off + en.end;
  return 0;
}

extern "C" void fls_st_close(void* h) { delete (StFile*)h; }
