// Pure C++ core of the host input-pipeline runtime (no Python): TFRecord framing with hardware
// CRC32C, bounds-checked tf.train.Example wire-format decoding, and the threaded uint8 NHWC ->
// float NCHW batch normalisation. Bound to Python by io.cpp (module deep_vision_amd._io) and
// compiled standalone with ASan/UBSan and TSan by io_selftest.cpp (tests/test_native_host.py):
// the sanitizers run on this host code only (GPU sanitizers are not available on the pool).
#pragma once

#include <nmmintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <sys/stat.h>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace dvio {

// ------------------------------------------------------------------ crc32c
inline uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0) {
  uint64_t c = ~crc & 0xffffffffu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
inline uint32_t masked_crc(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ------------------------------------------------------------------ record framing
// [u64 len][u32 masked crc32c(len)][data][u32 masked crc32c(data)]
inline void frame_header(uint64_t len, uint8_t hdr[12]) {
  std::memcpy(hdr, &len, 8);
  const uint32_t lc = masked_crc(hdr, 8);
  std::memcpy(hdr + 8, &lc, 4);
}

// Reads one record from f into out. false at a clean EOF; throws on truncation / bad CRC.
inline bool read_record(FILE* f, std::string& out, bool check, const std::string& path) {
  uint8_t hdr[12];
  const size_t got = std::fread(hdr, 1, 12, f);
  if (got == 0) return false;
  if (got != 12) throw std::runtime_error("truncated record header in " + path);
  uint64_t len;
  uint32_t lc;
  std::memcpy(&len, hdr, 8);
  std::memcpy(&lc, hdr + 8, 4);
  if (check && masked_crc(hdr, 8) != lc) throw std::runtime_error("corrupt record length (crc) in " + path);
  // bound the allocation by what the file can still hold (a corrupt length must not make
  // resize() ask for terabytes before the truncation check runs)
  const off_t here = ftello(f);
  struct stat sb;
  if (here < 0 || fstat(fileno(f), &sb) != 0) throw std::runtime_error("cannot stat " + path);
  const uint64_t remaining = sb.st_size > here ? uint64_t(sb.st_size - here) : 0;
  if (len > remaining || remaining - len < 4) throw std::runtime_error("truncated record in " + path);
  out.resize(len);
  if (len && std::fread(&out[0], 1, len, f) != len) throw std::runtime_error("truncated record in " + path);
  uint32_t dc;
  if (std::fread(&dc, 1, 4, f) != 4) throw std::runtime_error("truncated record footer in " + path);
  if (check && masked_crc((const uint8_t*)out.data(), len) != dc)
    throw std::runtime_error("corrupt record data (crc) in " + path);
  return true;
}

inline std::vector<int64_t> index_file(const std::string& path) {
  std::vector<int64_t> offs;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  int64_t pos = 0;
  for (;;) {
    uint8_t hdr[12];
    const size_t got = std::fread(hdr, 1, 12, f);
    if (got == 0) break;
    if (got != 12) { std::fclose(f); throw std::runtime_error("truncated record header in " + path); }
    uint64_t len;
    std::memcpy(&len, hdr, 8);
    offs.push_back(pos);
    pos += 12 + (int64_t)len + 4;
    if (fseeko(f, pos, SEEK_SET) != 0) break;
  }
  std::fclose(f);
  return offs;
}

// ------------------------------------------------------------------ Example decoding
// Every read is checked against the end of its enclosing message: a malformed or truncated
// Example throws instead of reading past the buffer (fuzzed under ASan by io_selftest.cpp).
struct Buf {
  const uint8_t* p;
  const uint8_t* e;
  size_t left() const { return (size_t)(e - p); }
  uint64_t varint() {
    uint64_t v = 0;
    int s = 0;
    while (p < e) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
      s += 7;
      if (s > 63) break;
    }
    throw std::runtime_error("malformed varint in Example");
  }
  void need(size_t n) const {
    if (left() < n) throw std::runtime_error("truncated Example field");
  }
  Buf sub() {
    const uint64_t n = varint();
    if (left() < n) throw std::runtime_error("truncated Example field");
    Buf b{p, p + n};
    p += n;
    return b;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) { need(8); p += 8; }
    else if (wt == 2) sub();
    else if (wt == 5) { need(4); p += 4; }
    else throw std::runtime_error("unsupported wire type in Example");
  }
};

enum class Kind { Empty, Bytes, Float, Int64 };
struct Feature {
  Kind kind = Kind::Empty;
  std::vector<std::string> bytes;
  std::vector<float> floats;
  std::vector<int64_t> ints;
};

// Feature { oneof { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
inline Feature decode_feature(Buf f) {
  Feature out;
  while (f.p < f.e) {
    const uint64_t key = f.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    if (wt != 2) { f.skip(wt); continue; }
    Buf l = f.sub();
    if (field == 1) {
      out.kind = Kind::Bytes;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) == 1 && (k & 7) == 2) {
          Buf s = l.sub();
          out.bytes.emplace_back((const char*)s.p, s.left());
        } else l.skip((int)(k & 7));
      }
      return out;
    }
    if (field == 2) {
      out.kind = Kind::Float;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) != 1) { l.skip((int)(k & 7)); continue; }
        if ((k & 7) == 2) {  // packed
          Buf s = l.sub();
          const size_t n = s.left() / 4;
          const size_t o = out.floats.size();
          out.floats.resize(o + n);
          if (n) std::memcpy(out.floats.data() + o, s.p, n * 4);
        } else if ((k & 7) == 5) {
          l.need(4);
          float x;
          std::memcpy(&x, l.p, 4);
          l.p += 4;
          out.floats.push_back(x);
        } else l.skip((int)(k & 7));
      }
      return out;
    }
    if (field == 3) {
      out.kind = Kind::Int64;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) != 1) { l.skip((int)(k & 7)); continue; }
        if ((k & 7) == 2) {
          Buf s = l.sub();
          while (s.p < s.e) out.ints.push_back((int64_t)s.varint());
        } else if ((k & 7) == 0) {
          out.ints.push_back((int64_t)l.varint());
        } else l.skip((int)(k & 7));
      }
      return out;
    }
  }
  return out;
}

// Example { Features features = 1; }  Features { map<string, Feature> feature = 1; }
inline std::vector<std::pair<std::string, Feature>> parse_example(const uint8_t* data, size_t n) {
  std::vector<std::pair<std::string, Feature>> out;
  Buf b{data, data + n};
  while (b.p < b.e) {
    const uint64_t key = b.varint();
    if ((key >> 3) != 1 || (key & 7) != 2) { b.skip((int)(key & 7)); continue; }
    Buf feats = b.sub();
    while (feats.p < feats.e) {
      const uint64_t k2 = feats.varint();
      if ((k2 >> 3) != 1 || (k2 & 7) != 2) { feats.skip((int)(k2 & 7)); continue; }
      Buf entry = feats.sub();  // map entry { string key = 1; Feature value = 2; }
      std::string name;
      Buf val{nullptr, nullptr};
      while (entry.p < entry.e) {
        const uint64_t k3 = entry.varint();
        const int fld = (int)(k3 >> 3);
        if ((k3 & 7) != 2) { entry.skip((int)(k3 & 7)); continue; }
        Buf x = entry.sub();
        if (fld == 1) name.assign((const char*)x.p, x.left());
        else if (fld == 2) val = x;
      }
      out.emplace_back(std::move(name), val.p ? decode_feature(val) : Feature{});
    }
  }
  return out;
}

// ------------------------------------------------------------------ batch normalisation
// src (N, H, W, C) uint8 -> dst (N, C, H, W) float32: (x / scale - mean[c]) / std[c]; rows of
// (n, h) split over `threads` workers, each writing a disjoint set of output rows.
inline void normalize_batch(const uint8_t* s, float* d, int64_t N, int64_t H, int64_t W, int64_t C,
                            const std::vector<float>& mean, const std::vector<float>& stdv, float scale, int threads) {
  if ((int64_t)mean.size() != C || (int64_t)stdv.size() != C) throw std::runtime_error("normalize_batch: mean/std size");
  std::vector<float> a(C), b(C);
  for (int64_t c = 0; c < C; ++c) { a[c] = 1.f / (scale * stdv[c]); b[c] = -mean[c] / stdv[c]; }
  const int64_t rows = N * H;
  if (rows <= 0) return;
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, rows));
  auto work = [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t n = r / H, h = r % H;
      const uint8_t* sp = s + r * W * C;
      for (int64_t c = 0; c < C; ++c) {
        float* dp = d + ((n * C + c) * H + h) * W;
        const float ac = a[c], bc = b[c];
        for (int64_t w = 0; w < W; ++w) dp[w] = sp[w * C + c] * ac + bc;
      }
    }
  };
  std::vector<std::thread> pool;
  const int64_t per = (rows + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t r0 = t * per, r1 = std::min(rows, r0 + per);
    if (r0 < r1) pool.emplace_back(work, r0, r1);
  }
  for (auto& th : pool) th.join();
}

// ---- image augmentation (the ImageNet train / val transforms, data/transforms.py) ----
// Rescale(shorter side -> S, new size truncated by int() like R/ResNet/pytorch/data_load.py:85-101)
// followed by a crop, computed in one pass for the crop window only: bilinear sampling with
// cv2.resize INTER_LINEAR's geometry (src = (dst + 0.5) * in/out - 0.5, clamped to the border, no
// antialiasing) -- the reference decodes and resizes with cv2 -- in 11-bit fixed point per axis
// like cv2's uint8 path. src: [H][W][C] uint8 with pixel stride ps >= C and row stride rs (a
// decoder's RGBX image read in place: ps = 4), dst: [ch][cw][C] contiguous.
inline void resize_crop_bilinear(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t outH, int64_t outW,
                                 int64_t cy, int64_t cx, int64_t ch, int64_t cw, uint8_t* dst, int64_t ps = 0,
                                 int64_t rs = 0) {
  if (H <= 0 || W <= 0 || outH <= 0 || outW <= 0 || cy < 0 || cx < 0 || cy + ch > outH || cx + cw > outW)
    throw std::runtime_error("resize_crop_bilinear: bad geometry");
  if (ps == 0) ps = C;
  if (rs == 0) rs = W * ps;
  if (ps < C || rs < W * ps) throw std::runtime_error("resize_crop_bilinear: bad strides");
  constexpr int BITS = 11, ONE = 1 << BITS;
  const double fy = (double)H / outH, fx = (double)W / outW;
  std::vector<int32_t> x0(cw), x1(cw), wx(cw);
  for (int64_t j = 0; j < cw; ++j) {
    double sx = (cx + j + 0.5) * fx - 0.5;
    if (sx < 0) sx = 0;
    int64_t a = (int64_t)sx;
    if (a > W - 1) a = W - 1;
    const double f = sx - a;
    x0[j] = (int32_t)(a * ps);
    x1[j] = (int32_t)(std::min<int64_t>(a + 1, W - 1) * ps);
    wx[j] = (int32_t)(f * ONE + 0.5);
  }
  for (int64_t i = 0; i < ch; ++i) {
    double sy = (cy + i + 0.5) * fy - 0.5;
    if (sy < 0) sy = 0;
    int64_t a = (int64_t)sy;
    if (a > H - 1) a = H - 1;
    const int32_t wy = (int32_t)((sy - a) * ONE + 0.5);
    const uint8_t* r0 = src + a * rs;
    const uint8_t* r1 = src + std::min<int64_t>(a + 1, H - 1) * rs;
    uint8_t* d = dst + i * cw * C;
    if (C == 3) {
      // RGB: channels unrolled, 32-bit sums (255 * 2^11 * 2^11 + 2^21 < 2^31: the same values as the
      // 64-bit form below), four taps' pointers hoisted per output pixel
      const int32_t wy1 = wy, wy0 = ONE - wy;
      for (int64_t j = 0; j < cw; ++j) {
        const int32_t w1 = wx[j], w0 = ONE - w1;
        const uint8_t *a0 = r0 + x0[j], *a1 = r0 + x1[j], *b0 = r1 + x0[j], *b1 = r1 + x1[j];
        uint8_t* o = d + j * 3;
        for (int c = 0; c < 3; ++c) {
          const int32_t top = a0[c] * w0 + a1[c] * w1, bot = b0[c] * w0 + b1[c] * w1;
          const int32_t v = (top * wy0 + bot * wy1 + (1 << (2 * BITS - 1))) >> (2 * BITS);
          o[c] = (uint8_t)(v > 255 ? 255 : v);
        }
      }
      continue;
    }
    for (int64_t j = 0; j < cw; ++j) {
      const int32_t w1 = wx[j], w0 = ONE - w1;
      for (int64_t c = 0; c < C; ++c) {
        const int32_t top = r0[x0[j] + c] * w0 + r0[x1[j] + c] * w1;
        const int32_t bot = r1[x0[j] + c] * w0 + r1[x1[j] + c] * w1;
        const int64_t v = ((int64_t)top * (ONE - wy) + (int64_t)bot * wy + ((int64_t)1 << (2 * BITS - 1))) >> (2 * BITS);
        d[j * C + c] = (uint8_t)(v > 255 ? 255 : v);
      }
    }
  }
}

// ColorJitter's PIL enhancers on an RGB uint8 [n][3] image, in place, in the given order
// (0 brightness, 1 contrast, 2 saturation; factors f[0..2], a factor of exactly 1 is skipped):
// each is Image.blend(degenerate, image, f) = degenerate + f * (image - degenerate), rounded and
// clipped to uint8 after every enhancer like PIL. Degenerates: black; the mean of the image's
// ITU-R 601-2 luma (L = (299 R + 587 G + 114 B) / 1000, rounded) as a flat gray; the per-pixel luma.
inline uint8_t clip_round(float v) {  // branch-free: the loops below vectorise
  return (uint8_t)(int)std::min(255.f, std::max(0.f, v));  // PIL ImagingBlend truncates
}
inline uint8_t luma(const uint8_t* p) { return (uint8_t)((p[0] * 19595 + p[1] * 38470 + p[2] * 7471 + 0x8000) >> 16); }
inline void color_jitter(uint8_t* img, int64_t n, const float* f, const int* order) {
  std::vector<float> g;
  for (int k = 0; k < 3; ++k) {
    const int op = order[k];
    const float a = f[op];
    if (a == 1.f) continue;
    if (op == 0) {
      for (int64_t i = 0; i < n * 3; ++i) img[i] = clip_round(img[i] * a);
    } else if (op == 1) {
      int64_t sum = 0;
      for (int64_t i = 0; i < n; ++i) sum += luma(img + 3 * i);
      const float m = (float)(int64_t)((double)sum / (double)n + 0.5);
      for (int64_t i = 0; i < n * 3; ++i) img[i] = clip_round(m + a * ((float)img[i] - m));
    } else {
      g.resize(n);
      for (int64_t i = 0; i < n; ++i) g[i] = (float)luma(img + 3 * i);
      for (int64_t i = 0; i < n; ++i) {
        uint8_t* p = img + 3 * i;
        p[0] = clip_round(g[i] + a * ((float)p[0] - g[i]));
        p[1] = clip_round(g[i] + a * ((float)p[1] - g[i]));
        p[2] = clip_round(g[i] + a * ((float)p[2] - g[i]));
      }
    }
  }
}

}  // namespace dvio
