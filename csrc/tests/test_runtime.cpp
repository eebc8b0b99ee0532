// Host-side unit test of the native runtime, built with AddressSanitizer +
// UBSan (and separately ThreadSanitizer) by tests/test_sanitizers.py.
// Exercises the multi-threaded pread/pwrite engine, the block gather, the
// safetensors header index (incl. malformed headers) and the weight streamer
// (persistent pread pool + pinned chunk ring + asynchronous copies, on its
// GPU-free host copy engine: ring wrap-around and slot reuse, O_DIRECT and its
// buffered fallback, fp32 -> fp16 pieces, pieces split across chunks) without a GPU.
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
  // ---- weight streamer on the host copy engine
  {
    // a "layer file": 3 MiB header gap, then raw fp16 pieces and one fp32 piece, odd sizes
    const uint64_t fsz = (26ull << 20) + 4096 * 3 + 777;
    std::vector<uint8_t> fb(fsz);
    for (uint64_t i = 0; i < fsz; ++i) fb[i] = (uint8_t)((i * 2246822519u) >> 11);
    const std::string lf = dir + "/fls_rt_layer.bin";
    CHECK(fls_pwrite_from(lf.c_str(), 0, fsz, fb.data(), 4, 1) == (int64_t)fsz);
    // fp32 piece at [20 MiB, 20 MiB + 4 MiB): finite values so the f16 rounding is well defined
    const uint64_t f32_off = 20ull << 20, f32_n = 4ull << 20;
    for (uint64_t e = 0; e < f32_n / 4; ++e) {
      float v = (float)((int)(e % 2001) - 1000) * 0.37f;
      std::memcpy(fb.data() + f32_off + 4 * e, &v, 4);
    }
    CHECK(fls_pwrite_from(lf.c_str(), f32_off, f32_n, fb.data() + f32_off, 2, 0) == (int64_t)f32_n);
    std::vector<fls_piece_t> pcs;
    uint64_t dst = 0;
    auto add = [&](uint64_t off, uint64_t n, int kind) {
      fls_piece_t p{off, n, dst, kind, 0};
      pcs.push_back(p);
      dst += kind ? n / 2 : n;
      dst = (dst + 255) / 256 * 256;
    };
    add(3ull << 20, (5ull << 20) + 123, 0);           // split over several 1 MiB chunks
    add((8ull << 20) + 4096, 4096 * 3 + 5, 0);        // small piece, packed with the next (gap read through)
    add((8ull << 20) + 4096 * 5, (11ull << 20) + 11, 0);
    add(f32_off, f32_n, 1);                           // fp32 -> fp16 on the host
    add(f32_off + f32_n + 64, fsz - (f32_off + f32_n + 64), 0);
    std::vector<uint8_t> want(dst, 0);
    for (const auto& p : pcs) {
      if (p.kind == 0) {
        std::memcpy(want.data() + p.dst_off, fb.data() + p.file_off, p.nbytes);
      } else {
        fls_f32_to_f16((const float*)(fb.data() + p.file_off), (uint16_t*)(want.data() + p.dst_off), p.nbytes / 4);
      }
    }
    for (int direct = 0; direct < 2; ++direct) {
      for (int chunks : {1, 2, 3}) {
        // 1 MiB chunks, 4 pread threads; copies delayed so a premature slot reuse would overlap them
        void* sh = fls_streamer_create_host(1u << 20, chunks, 4, direct, 50);
        CHECK(sh != nullptr);
        if (!sh) continue;
        for (int rep = 0; rep < 3; ++rep) {          // the ring keeps rotating across loads
          std::vector<uint8_t> got(dst, 0xCD);
          const int64_t r = fls_streamer_load(sh, lf.c_str(), pcs.data(), (int)pcs.size(), got.data(), nullptr);
          CHECK(r > 0);
          CHECK(fls_streamer_sync_host(sh) == 0);
          for (const auto& p : pcs) {
            const uint64_t n = p.kind ? p.nbytes / 2 : p.nbytes;
            CHECK(std::memcmp(got.data() + p.dst_off, want.data() + p.dst_off, n) == 0);
          }
        }
        double rs, ws;
        uint64_t rb, hb;
        int fb_n = -1;
        CHECK(fls_streamer_stats(sh, &rs, &ws, &rb, &hb, &fb_n) == 0);
        CHECK(rb > 0 && hb > 0 && fb_n >= 0);
        fls_streamer_destroy(sh);
      }
    }
    // a larger chunk with several pread granules per chunk (8 MiB granules, 20 MiB chunk)
    void* sh = fls_streamer_create_host(20u << 20, 2, 3, 0, 0);
    CHECK(sh != nullptr);
    if (sh) {
      std::vector<uint8_t> got(dst, 0);
      CHECK(fls_streamer_load(sh, lf.c_str(), pcs.data(), (int)pcs.size(), got.data(), nullptr) > 0);
      CHECK(fls_streamer_sync_host(sh) == 0);
      CHECK(std::memcmp(got.data(), want.data(), dst) == 0);
      // unsorted pieces and bad kinds are rejected
      fls_piece_t bad2[2] = {pcs[1], pcs[0]};
      CHECK(fls_streamer_load(sh, lf.c_str(), bad2, 2, got.data(), nullptr) < 0);
      fls_piece_t badk = pcs[0];
      badk.kind = 7;
      CHECK(fls_streamer_load(sh, lf.c_str(), &badk, 1, got.data(), nullptr) < 0);
      CHECK(fls_streamer_load(sh, (dir + "/missing.bin").c_str(), pcs.data(), 1, got.data(), nullptr) < 0);
      fls_streamer_destroy(sh);
    }
    CHECK(fls_streamer_create_host(1000, 2, 1, 0, 0) == nullptr);     // chunk below 1 MiB
    std::remove(lf.c_str());
  }
  std::remove(blob.c_str());
  std::remove(st.c_str());
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("runtime host test ok\n");
  return 0;
}
