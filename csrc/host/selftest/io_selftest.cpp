// Standalone self-test of the host input-pipeline core (csrc/host/io_core.h), built and run under
// AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer by
// tests/test_native_host.py (host code only: GPU sanitizers / xnack are not available here).
//   1. CRC32C against the standard check value;
//   2. TFRecord write -> index -> sequential and random-access read, CRC verification;
//   3. tf.train.Example decoding of a hand-encoded message, then a fuzz pass over every
//      truncation and 20k random byte mutations: malformed input must throw, never read out of
//      bounds (ASan) or hit UB (UBSan);
//   4. the threaded normalize_batch against a single-threaded run (TSan: no data race).
#include <cstdio>
#include <cstdlib>
#include <random>

#include <unistd.h>

#include "../io_core.h"

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) { s.push_back((char)(v | 0x80)); v >>= 7; }
  s.push_back((char)v);
}
static void put_ld(std::string& s, int field, const std::string& payload) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, payload.size());
  s += payload;
}

static std::string make_example() {
  std::string bytes_list, f_bytes, floats_packed, f_float, ints_packed, f_int, unpacked, f_unp;
  put_ld(bytes_list, 1, "hello");
  put_ld(bytes_list, 1, std::string("\x00\x01\x02", 3));
  put_ld(f_bytes, 1, bytes_list);
  std::string fl;
  const float vals[3] = {0.5f, -1.25f, 3.f};
  fl.append((const char*)vals, sizeof(vals));
  put_ld(floats_packed, 1, fl);
  put_ld(f_float, 2, floats_packed);
  std::string iv;
  for (int64_t v : {1, 300, 70000}) put_varint(iv, (uint64_t)v);
  put_ld(ints_packed, 1, iv);
  put_ld(f_int, 3, ints_packed);
  put_varint(unpacked, (1 << 3) | 5);  // unpacked float
  unpacked.append((const char*)&vals[1], 4);
  put_ld(f_unp, 2, unpacked);
  std::string feats;
  const std::pair<const char*, std::string*> entries[4] = {
      {"image/encoded", &f_bytes}, {"bbox", &f_float}, {"label", &f_int}, {"scalar", &f_unp}};
  for (auto& e : entries) {
    std::string entry;
    put_ld(entry, 1, e.first);
    put_ld(entry, 2, *e.second);
    put_ld(feats, 1, entry);
  }
  std::string ex;
  put_ld(ex, 1, feats);
  return ex;
}

int main() {
  // 1. crc32c check value
  const char* c9 = "123456789";
  CHECK(dvio::crc32c((const uint8_t*)c9, 9) == 0xE3069283u);

  // 2. TFRecord round trip
  const std::string path = "/tmp/dv_io_selftest_" + std::to_string((long)getpid()) + ".tfrecord";
  std::vector<std::string> recs;
  std::mt19937 rng(1234);
  for (int i = 0; i < 64; ++i) {
    std::string r(rng() % 5000, '\0');
    for (auto& ch : r) ch = (char)(rng() & 0xff);
    recs.push_back(r);
  }
  FILE* f = std::fopen(path.c_str(), "wb");
  CHECK(f);
  for (auto& r : recs) {
    uint8_t hdr[12];
    dvio::frame_header(r.size(), hdr);
    const uint32_t dc = dvio::masked_crc((const uint8_t*)r.data(), r.size());
    std::fwrite(hdr, 1, 12, f);
    std::fwrite(r.data(), 1, r.size(), f);
    std::fwrite(&dc, 1, 4, f);
  }
  std::fclose(f);
  auto offs = dvio::index_file(path);
  CHECK(offs.size() == recs.size());
  f = std::fopen(path.c_str(), "rb");
  std::string out;
  for (size_t i = 0; i < recs.size(); ++i) {
    CHECK(dvio::read_record(f, out, true, path));
    CHECK(out == recs[i]);
  }
  CHECK(!dvio::read_record(f, out, true, path));
  for (int i = (int)recs.size() - 1; i >= 0; i -= 7) {
    CHECK(fseeko(f, offs[i], SEEK_SET) == 0);
    CHECK(dvio::read_record(f, out, true, path) && out == recs[i]);
  }
  std::fclose(f);
  std::remove(path.c_str());

  // 3. Example decoding + fuzz
  const std::string ex = make_example();
  auto feats = dvio::parse_example((const uint8_t*)ex.data(), ex.size());
  CHECK(feats.size() == 4);
  CHECK(feats[0].first == "image/encoded" && feats[0].second.kind == dvio::Kind::Bytes);
  CHECK(feats[0].second.bytes.size() == 2 && feats[0].second.bytes[0] == "hello");
  CHECK(feats[1].second.kind == dvio::Kind::Float && feats[1].second.floats.size() == 3 &&
        feats[1].second.floats[1] == -1.25f);
  CHECK(feats[2].second.kind == dvio::Kind::Int64 && feats[2].second.ints[2] == 70000);
  CHECK(feats[3].second.floats.size() == 1 && feats[3].second.floats[0] == -1.25f);
  size_t thrown = 0, parsed = 0;
  for (size_t n = 0; n < ex.size(); ++n) {  // every truncation, in an exactly-sized heap buffer
    std::vector<uint8_t> buf(ex.begin(), ex.begin() + n);
    try { dvio::parse_example(buf.data(), buf.size()); ++parsed; } catch (const std::exception&) { ++thrown; }
  }
  for (int it = 0; it < 20000; ++it) {
    std::vector<uint8_t> buf(ex.begin(), ex.end());
    const int flips = 1 + (int)(rng() % 4);
    for (int k = 0; k < flips; ++k) buf[rng() % buf.size()] = (uint8_t)(rng() & 0xff);
    buf.resize(rng() % (buf.size() + 1));
    try { dvio::parse_example(buf.data(), buf.size()); ++parsed; } catch (const std::exception&) { ++thrown; }
  }
  CHECK(thrown > 0 && parsed > 0);

  // 4. threaded normalisation == single-threaded
  const int64_t N = 3, H = 37, W = 29, C = 3;
  std::vector<uint8_t> img(N * H * W * C);
  for (auto& v : img) v = (uint8_t)(rng() & 0xff);
  std::vector<float> a(N * C * H * W), b(N * C * H * W);
  const std::vector<float> mean = {0.485f, 0.456f, 0.406f}, stdv = {0.229f, 0.224f, 0.225f};
  dvio::normalize_batch(img.data(), a.data(), N, H, W, C, mean, stdv, 255.f, 1);
  dvio::normalize_batch(img.data(), b.data(), N, H, W, C, mean, stdv, 255.f, 8);
  CHECK(a == b);
  CHECK(std::abs(a[0] - ((img[0] / 255.f - mean[0]) / stdv[0])) < 1e-5f);
  std::printf("io_selftest ok: %zu records, fuzz %zu parsed / %zu rejected\n", recs.size(), parsed, thrown);
  return 0;
}
