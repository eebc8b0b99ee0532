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
//   scanner specialised for the format;
// * the weight streamer: per-layer file byte ranges -> a ring of pinned chunk
//   buffers (persistent pread pool, optional O_DIRECT) -> hipMemcpyAsync of
//   every tensor piece straight to its place in the HBM weight slot, on the
//   caller's copy stream (reference: read + deserialize + per-tensor pageable
//   H2D, utils.py:121-131).
//
// Built with g++ against libamdhip64 (host code only).
#include "fls.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
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
  // portable: the same pinned block may feed H2D copies of any device of the process
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocPortable);
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

// device address of a mapped pinned host block (hipHostMalloc): kernels read / write it over PCIe
// (runtime/prefix_cache.py host mode writes a generation step's new K/V rows straight into it);
// nullptr when the block is not mapped
extern "C" void* fls_host_device_ptr(void* p) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
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

// exact-size device allocations outside PyTorch's caching allocator (weight slots: allocated
// once per run, never split or cached per stream)
extern "C" void* fls_device_alloc(int device, uint64_t bytes) {
  void* p = nullptr;
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

extern "C" int fls_device_free(int device, void* p) {
  if (!p) return 0;
  (void)hipSetDevice(device);
  return hipFree(p) == hipSuccess ? 0 : -1;
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

// ------------------------------------------------------------- streamer
namespace {

// fp32 -> fp16 bits, round to nearest even, overflow -> inf, NaN kept (torch .to(float16))
inline uint16_t f32_to_f16_bits(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7FFFFFFFu;
  if (ax >= 0x7F800000u) return (uint16_t)(sign | 0x7C00u | (ax > 0x7F800000u ? 0x200u : 0u));
  if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);          // rounds past 65504 -> inf
  if (ax < 0x38800000u) {                                            // fp16 subnormal or zero
    if (ax < 0x33000000u) return (uint16_t)sign;                     // < 2^-25: rounds to 0
    const uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;
    const int shift = 126 - (int)(ax >> 23);                         // 14 .. 24
    const uint32_t r = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    return (uint16_t)(sign | (r + (rem > half || (rem == half && (r & 1)))));
  }
  const uint32_t r = ((ax - 0x38000000u) >> 13), rem = ax & 0x1FFFu;
  return (uint16_t)(sign | (r + (rem > 0x1000u || (rem == 0x1000u && (r & 1)))));
}

// persistent worker pool for parallel pread granules
class IoPool {
 public:
  explicit IoPool(int n) {
    for (int i = 0; i < std::max(1, n); ++i) ts_.emplace_back([this] { loop(); });
  }
  ~IoPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : ts_) t.join();
  }
  // run f(0..n-1) on the pool, return when all are done
  void run(int64_t n, const std::function<void(int64_t)>& f) {
    if (n <= 0) return;
    std::unique_lock<std::mutex> g(m_);
    job_ = &f;
    n_ = n;
    next_ = 0;
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(g, [&] { return done_ == n_; });
    job_ = nullptr;
  }
  int size() const { return (int)ts_.size(); }

 private:
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || (gen_ != seen && job_ && next_ < n_); });
      if (stop_) return;
      while (job_ && next_ < n_) {
        const int64_t i = next_++;
        const std::function<void(int64_t)>* f = job_;
        g.unlock();
        (*f)(i);
        g.lock();
        if (++done_ == n_) done_cv_.notify_all();
      }
      seen = gen_;
    }
  }
  std::vector<std::thread> ts_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* job_ = nullptr;
  int64_t n_ = 0, next_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// The streamer's device side behind an interface: HIP in production; a host engine (malloc'd
// ring, copies run by a worker thread in FIFO order, events signalled by that thread) so the
// ring's slot reuse, the pread pool and the O_DIRECT fallback run under ASan / TSan without a
// GPU (csrc/tests/test_runtime.cpp).  The host engine's copies READ the ring slot
// asynchronously exactly as the DMA engine does, so reusing a slot before its event fired is a
// data race TSan reports (and a wrong byte the test sees).
struct CopyEngine {
  virtual ~CopyEngine() = default;
  virtual int set_device() = 0;
  virtual void* alloc_host(uint64_t n) = 0;
  virtual void free_host(void* p) = 0;
  virtual void* event_create() = 0;
  virtual void event_destroy(void* ev) = 0;
  virtual int event_record(void* ev, void* stream) = 0;
  virtual int event_sync(void* ev) = 0;
  virtual int copy_async(void* dst, const void* src, uint64_t n, void* stream) = 0;
};

struct HipEngine final : CopyEngine {
  int device;
  explicit HipEngine(int d) : device(d) {}
  int set_device() override {
    if (hipSetDevice(device) != hipSuccess) { (void)hipGetLastError(); return -1; }
    return 0;
  }
  void* alloc_host(uint64_t n) override {
    void* p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocPortable) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
    return p;
  }
  void free_host(void* p) override { (void)hipHostFree(p); }
  void* event_create() override {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
    return ev;
  }
  void event_destroy(void* ev) override { (void)hipEventDestroy((hipEvent_t)ev); }
  int event_record(void* ev, void* stream) override {
    if (hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) != hipSuccess) { (void)hipGetLastError(); return -1; }
    return 0;
  }
  int event_sync(void* ev) override {
    if (hipEventSynchronize((hipEvent_t)ev) != hipSuccess) { (void)hipGetLastError(); return -1; }
    return 0;
  }
  int copy_async(void* dst, const void* src, uint64_t n, void* stream) override {
    if (hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    return 0;
  }
};

struct HostEngine final : CopyEngine {
  struct Ev {
    uint64_t recorded = 0, done = 0;
  };
  struct Task {
    void* dst;
    const void* src;
    uint64_t n;
    Ev* ev;
    uint64_t gen;
  };
  std::mutex m;
  std::condition_variable cv, done_cv;
  std::deque<Task> q;
  bool busy = false;
  bool stop = false;
  int delay_us;
  std::thread worker;
  explicit HostEngine(int delay) : delay_us(delay) { worker = std::thread([this] { loop(); }); }
  ~HostEngine() override {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    worker.join();
  }
  void loop() {
    std::unique_lock<std::mutex> g(m);
    for (;;) {
      cv.wait(g, [&] { return stop || !q.empty(); });
      if (q.empty()) return;   // stop requested and nothing left
      Task t = q.front();
      q.pop_front();
      busy = true;
      g.unlock();
      if (t.ev == nullptr) {
        if (delay_us) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
        std::memcpy(t.dst, t.src, t.n);           // the "DMA" reads the pinned slot now
      }
      g.lock();
      busy = false;
      if (t.ev) t.ev->done = t.gen;
      done_cv.notify_all();
    }
  }
  int set_device() override { return 0; }
  void* alloc_host(uint64_t n) override { return std::malloc(n); }
  void free_host(void* p) override { std::free(p); }
  void* event_create() override { return new Ev(); }
  void event_destroy(void* ev) override { delete (Ev*)ev; }
  int event_record(void* ev, void*) override {
    std::lock_guard<std::mutex> g(m);
    Ev* e = (Ev*)ev;
    q.push_back({nullptr, nullptr, 0, e, ++e->recorded});
    cv.notify_all();
    return 0;
  }
  int event_sync(void* ev) override {
    std::unique_lock<std::mutex> g(m);
    Ev* e = (Ev*)ev;
    done_cv.wait(g, [&] { return e->done >= e->recorded; });
    return 0;
  }
  int copy_async(void* dst, const void* src, uint64_t n, void*) override {
    std::lock_guard<std::mutex> g(m);
    q.push_back({dst, src, n, nullptr, 0});
    cv.notify_all();
    return 0;
  }
  void drain() {
    std::unique_lock<std::mutex> g(m);
    done_cv.wait(g, [&] { return q.empty() && !busy; });
  }
};

struct Slot {
  char* buf = nullptr;
  void* ev = nullptr;
  bool pending = false;
};

struct Streamer {
  CopyEngine* eng = nullptr;
  bool host = false;
  uint64_t chunk = 0;
  int direct = 0;
  std::vector<Slot> slots;
  size_t next = 0;
  IoPool* pool = nullptr;
  // stats
  double read_s = 0, wait_s = 0;
  uint64_t read_bytes = 0, h2d_bytes = 0;
  int direct_fallbacks = 0;
};

struct SubPiece {
  uint64_t file_off, nbytes, dst_off;
  int kind;
};

constexpr uint64_t kAlign = 4096;
constexpr uint64_t kGranule = 8ull << 20;   // pread granule per pool task

// read [lo, hi) of fd into buf (buf corresponds to file offset lo); returns 0 or -errno
int64_t pool_read(IoPool* pool, int fd, uint64_t lo, uint64_t hi, char* buf, uint64_t need_hi) {
  const uint64_t bytes = hi - lo;
  const int64_t n = (int64_t)((bytes + kGranule - 1) / kGranule);
  std::atomic<int64_t> err{0};
  pool->run(n, [&](int64_t c) {
    const uint64_t a = (uint64_t)c * kGranule, len = std::min<uint64_t>(kGranule, bytes - a);
    uint64_t done = 0;
    while (done < len) {
      ssize_t r = pread(fd, buf + a + done, len - done, lo + a + done);
      if (r < 0) {
        if (errno == EINTR) continue;
        err.store(-errno);
        return;
      }
      if (r == 0) {   // EOF: fine past the bytes we need (O_DIRECT rounds the range up)
        if (lo + a + done < need_hi) err.store(-EIO);
        return;
      }
      done += (uint64_t)r;
    }
  });
  return err.load();
}

}  // namespace

static Streamer* streamer_new(CopyEngine* eng, bool host, uint64_t chunk_bytes, int n_chunks, int io_threads,
                              int direct) {
  if (chunk_bytes < (1u << 20) || n_chunks < 1 || eng->set_device() != 0) {
    delete eng;
    return nullptr;
  }
  auto* st = new Streamer();
  st->eng = eng;
  st->host = host;
  st->chunk = (chunk_bytes + kAlign - 1) / kAlign * kAlign;
  st->direct = direct;
  st->slots.resize(n_chunks);
  for (auto& sl : st->slots) {
    // + 2 alignment pages: an O_DIRECT read rounds the range out on both sides
    void* p = eng->alloc_host(st->chunk + 2 * kAlign);
    void* ev = p ? eng->event_create() : nullptr;
    if (!p || !ev) {
      if (p) eng->free_host(p);
      for (auto& s2 : st->slots) {
        if (s2.buf) eng->free_host(s2.buf);
        if (s2.ev) eng->event_destroy(s2.ev);
      }
      delete eng;
      delete st;
      return nullptr;
    }
    sl.buf = (char*)p;
    sl.ev = ev;
  }
  st->pool = new IoPool(std::max(1, io_threads));
  return st;
}

extern "C" void* fls_streamer_create(int device, uint64_t chunk_bytes, int n_chunks, int io_threads, int direct) {
  return streamer_new(new HipEngine(device), false, chunk_bytes, n_chunks, io_threads, direct);
}

// GPU-free streamer (tests, sanitizers): `dst_dev` of fls_streamer_load is a host pointer, copies
// are done by a worker thread (each optionally delayed by copy_delay_us to widen race windows)
extern "C" void* fls_streamer_create_host(uint64_t chunk_bytes, int n_chunks, int io_threads, int direct,
                                          int copy_delay_us) {
  return streamer_new(new HostEngine(copy_delay_us), true, chunk_bytes, n_chunks, io_threads, direct);
}

// host streamer: wait until every enqueued copy is done
extern "C" int fls_streamer_sync_host(void* h) {
  auto* st = (Streamer*)h;
  if (!st || !st->host) return -1;
  static_cast<HostEngine*>(st->eng)->drain();
  return 0;
}

extern "C" uint64_t fls_streamer_pinned_bytes(void* h) {
  auto* st = (Streamer*)h;
  return st ? (uint64_t)st->slots.size() * (st->chunk + 2 * kAlign) : 0;
}

// Stream `n` pieces of `path` (sorted by file_off) to dst_dev + piece.dst_off on `stream`.
// kind 0: raw bytes; kind 1: fp32 source converted to fp16 on the host (nbytes fp32 bytes in
// the file, nbytes / 2 bytes written).  Returns the file bytes read, or < 0 on error.  Returns
// once every copy is ENQUEUED; the caller records its own completion event on `stream`.
extern "C" int64_t fls_streamer_load(void* h, const char* path, const fls_piece_t* pieces, int n, void* dst_dev,
                                     fls_stream_t stream) {
  auto* st = (Streamer*)h;
  if (!st || n < 0) return -EINVAL;
  if (n == 0) return 0;
  if (st->eng->set_device() != 0) return -ENODEV;
  // split pieces so that every chunk (with O_DIRECT slack) fits a ring slot
  const uint64_t maxp = st->chunk;
  std::vector<SubPiece> sub;
  for (int i = 0; i < n; ++i) {
    const fls_piece_t& p = pieces[i];
    if (i && p.file_off < pieces[i - 1].file_off) return -EINVAL;
    if (p.kind != 0 && p.kind != 1) return -EINVAL;
    uint64_t a = 0;
    while (a < p.nbytes) {
      const uint64_t len = std::min<uint64_t>(maxp, p.nbytes - a);   // maxp % 4096 == 0: fp32 elements stay whole
      sub.push_back({p.file_off + a, len, p.dst_off + (p.kind == 1 ? a / 2 : a), (int)p.kind});
      a += len;
    }
  }
  int flags = O_RDONLY | O_CLOEXEC;
  int fd = -1;
  bool direct = st->direct != 0;
  if (direct) {
    fd = open(path, flags | O_DIRECT);
    if (fd < 0) { direct = false; ++st->direct_fallbacks; }
  }
  if (fd < 0) fd = open(path, flags);
  if (fd < 0) return -errno;
  if (!direct) posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  int64_t total = 0;
  size_t i = 0;
  while (i < sub.size()) {
    // chunk = consecutive sub-pieces whose file span fits the slot (small gaps are read through)
    const uint64_t lo = sub[i].file_off;
    size_t j = i + 1;
    uint64_t hi = sub[i].file_off + sub[i].nbytes;
    while (j < sub.size() && sub[j].file_off >= hi && sub[j].file_off - hi <= (1u << 20) &&
           sub[j].file_off + sub[j].nbytes - lo <= maxp) {
      hi = sub[j].file_off + sub[j].nbytes;
      ++j;
    }
    Slot& sl = st->slots[st->next++ % st->slots.size()];
    auto t0 = std::chrono::steady_clock::now();
    if (sl.pending) {
      if (st->eng->event_sync(sl.ev) != 0) { close(fd); return -EIO; }
      sl.pending = false;
    }
    auto t1 = std::chrono::steady_clock::now();
    uint64_t rlo = lo, rhi = hi;
    if (direct) {
      rlo = lo / kAlign * kAlign;
      rhi = (hi + kAlign - 1) / kAlign * kAlign;
    }
    int64_t r = pool_read(st->pool, fd, rlo, rhi, sl.buf, hi);
    if (r == -EINVAL && direct) {
      // the file system refused O_DIRECT for this range: buffered from here on
      close(fd);
      fd = open(path, flags);
      if (fd < 0) return -errno;
      direct = false;
      ++st->direct_fallbacks;
      rlo = lo;
      rhi = hi;
      r = pool_read(st->pool, fd, rlo, rhi, sl.buf, hi);
    }
    if (r < 0) { close(fd); return r; }
    auto t2 = std::chrono::steady_clock::now();
    st->wait_s += std::chrono::duration<double>(t1 - t0).count();
    st->read_s += std::chrono::duration<double>(t2 - t1).count();
    st->read_bytes += hi - lo;
    total += (int64_t)(hi - lo);
    for (size_t k = i; k < j; ++k) {
      char* src = sl.buf + (sub[k].file_off - rlo);
      uint64_t len = sub[k].nbytes;
      if (sub[k].kind == 1) {   // fp32 -> fp16 in place (write index <= read index: forward is safe)
        const uint64_t cnt = len / 4;
        const float* fs = (const float*)src;
        uint16_t* hs = (uint16_t*)src;
        for (uint64_t e = 0; e < cnt; ++e) {
          float v;
          std::memcpy(&v, fs + e, 4);
          hs[e] = f32_to_f16_bits(v);
        }
        len = cnt * 2;
      }
      if (st->eng->copy_async((char*)dst_dev + sub[k].dst_off, src, len, stream) != 0) {
        close(fd);
        return -EIO;
      }
      st->h2d_bytes += len;
    }
    if (st->eng->event_record(sl.ev, stream) != 0) { close(fd); return -EIO; }
    sl.pending = true;
    i = j;
  }
  close(fd);
  return total;
}

// host-only variant (no GPU): the same piece plan read into a host buffer (CPU runs / tests)
extern "C" int64_t fls_stream_read_host(const char* path, const fls_piece_t* pieces, int n, void* dst,
                                        int io_threads) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    const fls_piece_t& p = pieces[i];
    char* d = (char*)dst + p.dst_off;
    if (p.kind == 0) {
      int64_t r = parallel_io(fd, p.file_off, p.nbytes, d, io_threads, false);
      if (r < 0) { close(fd); return r; }
    } else {
      std::vector<char> tmp(p.nbytes);
      int64_t r = parallel_io(fd, p.file_off, p.nbytes, tmp.data(), io_threads, false);
      if (r < 0) { close(fd); return r; }
      const uint64_t cnt = p.nbytes / 4;
      for (uint64_t e = 0; e < cnt; ++e) {
        float v;
        std::memcpy(&v, tmp.data() + 4 * e, 4);
        const uint16_t b = f32_to_f16_bits(v);
        std::memcpy(d + 2 * e, &b, 2);
      }
    }
    total += (int64_t)p.nbytes;
  }
  close(fd);
  return total;
}

extern "C" int fls_streamer_stats(void* h, double* read_s, double* wait_s, uint64_t* read_bytes,
                                  uint64_t* h2d_bytes, int* direct_fallbacks) {
  auto* st = (Streamer*)h;
  if (!st) return -1;
  *read_s = st->read_s;
  *wait_s = st->wait_s;
  *read_bytes = st->read_bytes;
  *h2d_bytes = st->h2d_bytes;
  *direct_fallbacks = st->direct_fallbacks;
  return 0;
}

extern "C" void fls_streamer_destroy(void* h) {
  auto* st = (Streamer*)h;
  if (!st) return;
  (void)st->eng->set_device();
  for (auto& sl : st->slots) {
    if (sl.pending) (void)st->eng->event_sync(sl.ev);
    st->eng->event_destroy(sl.ev);
    st->eng->free_host(sl.buf);
  }
  delete st->pool;
  delete st->eng;
  delete st;
}

// host-only f32 -> f16 conversion with the streamer's rounding (tests)
extern "C" void fls_f32_to_f16(const float* src, uint16_t* dst, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) dst[i] = f32_to_f16_bits(src[i]);
}
