// Host-side unit test of the native runtime, built with AddressSanitizer +
// UBSan (and separately ThreadSanitizer) by tests/test_sanitizers.py.
// Exercises the multi-threaded pread/pwrite engine, the block gather and the
// safetensors header index (incl. malformed headers) without a GPU.
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fls.h"

static int fails = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                        \
    }                                                                 \
  } while (0)

static void write_file(const std::string& p, const std::string& data) {
  FILE* f = std::fopen(p.c_str(), "wb");
  std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // ---- pwrite / pread, several chunks and threads, odd sizes
  const uint64_t n = (40ull << 20) + 12345;
  std::vector<uint8_t> src(n), dst(n, 0);
  for (uint64_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
  const std::string blob = dir + "/fls_rt_blob.bin";
  CHECK(fls_pwrite_from(blob.c_str(), 0, n, src.data(), 7, 1) == (int64_t)n);
  CHECK(fls_pread_into(blob.c_str(), 0, n, dst.data(), 5) == (int64_t)n);
  CHECK(std::memcmp(src.data(), dst.data(), n) == 0);
  std::vector<uint8_t> part(777);
  CHECK(fls_pread_into(blob.c_str(), 1000001, 777, part.data(), 3) == 777);
  CHECK(std::memcmp(part.data(), src.data() + 1000001, 777) == 0);
  // reading past EOF is an error, not a hang or overflow
  CHECK(fls_pread_into(blob.c_str(), n - 10, 100, part.data(), 2) < 0);
  CHECK(fls_pread_into((dir + "/does_not_exist").c_str(), 0, 10, part.data(), 1) < 0);

  // ---- block gather
  std::vector<int32_t> a(64), b(64);
  for (int i = 0; i < 64; ++i) a[i] = i;
  int64_t perm[8] = {7, 6, 5, 4, 3, 2, 1, 0};
  fls_gather_blocks(b.data(), a.data(), 32, perm, 8, 4);
  for (int blk = 0; blk < 8; ++blk)
    for (int j = 0; j < 8; ++j) CHECK(b[blk * 8 + j] == a[perm[blk] * 8 + j]);

  // ---- safetensors header index
  std::string hdr =
      "{\"__metadata__\":{\"format\":\"pt\"},\"x.weight\":{\"dtype\":\"F16\",\"shape\":[2,3],"
      "\"data_offsets\":[0,12]},\"y\":{\"dtype\":\"F32\",\"shape\":[],\"data_offsets\":[12,16]}}";
  while (hdr.size() % 8) hdr += ' ';
  uint64_t hl = hdr.size();
  std::string file(reinterpret_cast<const char*>(&hl), 8);
  file += hdr + std::string(16, '\x01');
  const std::string st = dir + "/fls_rt_test.safetensors";
  write_file(st, file);
  void* h = fls_st_open(st.c_str());
  CHECK(h != nullptr);
  if (h) {
    CHECK(fls_st_count(h) == 2);
    char name[64], dt[16];
    int64_t shape[8];
    int nd = -1;
    uint64_t be = 0, en = 0;
    CHECK(fls_st_info(h, 0, name, 64, dt, 16, shape, &nd, &be, &en) == 0);
    CHECK(std::string(name) == "x.weight" && std::string(dt) == "F16" && nd == 2 && shape[1] == 3);
    CHECK(be == 8 + hl && en == 8 + hl + 12);
    CHECK(fls_st_info(h, 1, name, 64, dt, 16, shape, &nd, &be, &en) == 0 && nd == 0);
    CHECK(fls_st_info(h, 2, name, 64, dt, 16, shape, &nd, &be, &en) != 0);
    CHECK(fls_st_info(h, 0, name, 3, dt, 16, shape, &nd, &be, &en) != 0);   // name buffer too small
    fls_st_close(h);
  }
  // malformed headers must be rejected cleanly
  const char* bad[] = {"{\"a\":{\"dtype\":\"F16\",\"shape\":[1,", "{\"a\" \"b\"}", "[1,2,3]", "{\"a\":{\"shape\":[1}}"};
  for (const char* bh : bad) {
    std::string s(bh);
    uint64_t l = s.size();
    std::string f2(reinterpret_cast<const char*>(&l), 8);
    f2 += s;
    write_file(st, f2);
    void* hb = fls_st_open(st.c_str());
    CHECK(hb == nullptr);
    if (hb) fls_st_close(hb);
  }
  // absurd header length
  uint64_t huge = 1ull << 40;
  write_file(st, std::string(reinterpret_cast<const char*>(&huge), 8));
  CHECK(fls_st_open(st.c_str()) == nullptr);
  std::remove(blob.c_str());
  std::remove(st.c_str());
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("runtime host test ok\n");
  return 0;
}
