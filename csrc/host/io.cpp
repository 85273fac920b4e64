// Host-side native runtime of the input pipeline (module deep_vision_amd._io, no GPU code).
//
//  * TFRecord framing (TF-free): [u64 len][u32 masked crc32c(len)][data][u32 masked crc32c(data)]
//    with hardware CRC32C (SSE4.2 crc32 instruction, 8 bytes/cycle) -- RecordWriter,
//    RecordReader (sequential, or random access through an offset index so a sampler can
//    shuffle records), index_file.
//  * tf.train.Example decoding straight from the protobuf wire format (Features map of
//    BytesList / FloatList / Int64List, packed or unpacked) into Python lists: the per-record
//    hot path of every TFRecord dataset.
//  * normalize_batch: uint8 NHWC images -> float32 NCHW (x/scale - mean)/std over a thread pool
//    (the collate step of the ImageNet loader, R/ResNet/pytorch/data_load.py:176-210).
//
// The GIL is released around file IO and the pixel loop.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <nmmintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

// ------------------------------------------------------------------ crc32c
static uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0) {
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
static uint32_t masked_crc(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ------------------------------------------------------------------ writer
class RecordWriter {
 public:
  explicit RecordWriter(const std::string& path) {
    f_ = std::fopen(path.c_str(), "wb");
    if (!f_) throw std::runtime_error("cannot open " + path + " for writing");
  }
  ~RecordWriter() { close(); }
  void write(py::bytes b) {
    if (!f_) throw std::runtime_error("writer closed");
    std::string s = b;
    const uint64_t len = s.size();
    uint8_t hdr[12];
    std::memcpy(hdr, &len, 8);
    const uint32_t lc = masked_crc(hdr, 8);
    std::memcpy(hdr + 8, &lc, 4);
    const uint32_t dc = masked_crc((const uint8_t*)s.data(), s.size());
    py::gil_scoped_release nogil;
    std::fwrite(hdr, 1, 12, f_);
    std::fwrite(s.data(), 1, s.size(), f_);
    std::fwrite(&dc, 1, 4, f_);
  }
  void flush() { if (f_) std::fflush(f_); }
  void close() {
    if (f_) { std::fclose(f_); f_ = nullptr; }
  }

 private:
  FILE* f_ = nullptr;
};

// ------------------------------------------------------------------ reader
class RecordReader {
 public:
  RecordReader(const std::string& path, bool check_crc) : path_(path), check_(check_crc) {
    f_ = std::fopen(path.c_str(), "rb");
    if (!f_) throw std::runtime_error("cannot open " + path);
  }
  ~RecordReader() { if (f_) std::fclose(f_); }

  // next record or None at EOF
  py::object next() {
    std::string out;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = read_one(out);
    }
    if (!ok) return py::none();
    return py::bytes(out);
  }
  py::bytes read_at(int64_t offset) {
    std::string out;
    bool ok;
    {
      py::gil_scoped_release nogil;
      if (fseeko(f_, offset, SEEK_SET) != 0) throw std::runtime_error("seek failed in " + path_);
      ok = read_one(out);
    }
    if (!ok) throw std::runtime_error("no record at offset " + std::to_string(offset) + " in " + path_);
    return py::bytes(out);
  }
  void reset() { fseeko(f_, 0, SEEK_SET); }

 private:
  bool read_one(std::string& out) {
    uint8_t hdr[12];
    const size_t got = std::fread(hdr, 1, 12, f_);
    if (got == 0) return false;
    if (got != 12) throw std::runtime_error("truncated record header in " + path_);
    uint64_t len;
    uint32_t lc;
    std::memcpy(&len, hdr, 8);
    std::memcpy(&lc, hdr + 8, 4);
    if (check_ && masked_crc(hdr, 8) != lc) throw std::runtime_error("corrupt record length (crc) in " + path_);
    out.resize(len);
    if (len && std::fread(&out[0], 1, len, f_) != len) throw std::runtime_error("truncated record in " + path_);
    uint32_t dc;
    if (std::fread(&dc, 1, 4, f_) != 4) throw std::runtime_error("truncated record footer in " + path_);
    if (check_ && masked_crc((const uint8_t*)out.data(), len) != dc)
      throw std::runtime_error("corrupt record data (crc) in " + path_);
    return true;
  }
  std::string path_;
  bool check_;
  FILE* f_ = nullptr;
};

static std::vector<int64_t> index_file(const std::string& path) {
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
struct Buf {
  const uint8_t* p;
  const uint8_t* e;
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
  Buf sub() {
    const uint64_t n = varint();
    if ((uint64_t)(e - p) < n) throw std::runtime_error("truncated Example field");
    Buf b{p, p + n};
    p += n;
    return b;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) p += 8;
    else if (wt == 2) sub();
    else if (wt == 5) p += 4;
    else throw std::runtime_error("unsupported wire type in Example");
  }
};

static py::object decode_list(Buf f) {
  // Feature { oneof { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
  while (f.p < f.e) {
    const uint64_t key = f.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    if (wt != 2) { f.skip(wt); continue; }
    Buf l = f.sub();
    if (field == 1) {
      py::list out;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) == 1 && (k & 7) == 2) {
          Buf s = l.sub();
          out.append(py::bytes((const char*)s.p, s.e - s.p));
        } else l.skip((int)(k & 7));
      }
      return py::make_tuple("bytes", out);
    }
    if (field == 2) {
      std::vector<float> v;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) != 1) { l.skip((int)(k & 7)); continue; }
        if ((k & 7) == 2) {  // packed
          Buf s = l.sub();
          const size_t n = (s.e - s.p) / 4;
          const size_t o = v.size();
          v.resize(o + n);
          std::memcpy(v.data() + o, s.p, n * 4);
        } else if ((k & 7) == 5) {
          float x;
          std::memcpy(&x, l.p, 4);
          l.p += 4;
          v.push_back(x);
        } else l.skip((int)(k & 7));
      }
      return py::make_tuple("float", py::cast(v));
    }
    if (field == 3) {
      std::vector<int64_t> v;
      while (l.p < l.e) {
        const uint64_t k = l.varint();
        if ((k >> 3) != 1) { l.skip((int)(k & 7)); continue; }
        if ((k & 7) == 2) {
          Buf s = l.sub();
          while (s.p < s.e) v.push_back((int64_t)s.varint());
        } else if ((k & 7) == 0) {
          v.push_back((int64_t)l.varint());
        } else l.skip((int)(k & 7));
      }
      return py::make_tuple("int64", py::cast(v));
    }
  }
  return py::make_tuple("empty", py::list());
}

// Example { Features features = 1; }  Features { map<string, Feature> feature = 1; }
static py::dict parse_example(py::bytes data) {
  std::string s = data;
  Buf b{(const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size()};
  py::dict out;
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
        if (fld == 1) name.assign((const char*)x.p, x.e - x.p);
        else if (fld == 2) val = x;
      }
      out[py::str(name)] = val.p ? decode_list(val) : py::make_tuple("empty", py::list());
    }
  }
  return out;
}

// ------------------------------------------------------------------ batch normalisation
static void normalize_batch(py::array_t<uint8_t, py::array::c_style> src, py::array_t<float, py::array::c_style> dst,
                            std::vector<float> mean, std::vector<float> stdv, float scale, int threads) {
  // src (N, H, W, C) uint8 -> dst (N, C, H, W) float32: (x / scale - mean[c]) / std[c]
  if (src.ndim() != 4 || dst.ndim() != 4) throw std::runtime_error("normalize_batch: 4-D arrays expected");
  const int64_t N = src.shape(0), H = src.shape(1), W = src.shape(2), C = src.shape(3);
  if (dst.shape(0) != N || dst.shape(1) != C || dst.shape(2) != H || dst.shape(3) != W)
    throw std::runtime_error("normalize_batch: dst must be (N, C, H, W)");
  if ((int64_t)mean.size() != C || (int64_t)stdv.size() != C) throw std::runtime_error("normalize_batch: mean/std size");
  const uint8_t* s = src.data();
  float* d = dst.mutable_data();
  std::vector<float> a(C), b(C);
  for (int64_t c = 0; c < C; ++c) { a[c] = 1.f / (scale * stdv[c]); b[c] = -mean[c] / stdv[c]; }
  const int64_t rows = N * H;
  threads = std::max(1, std::min<int>(threads, (int)rows));
  py::gil_scoped_release nogil;
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

PYBIND11_MODULE(_io, m) {
  m.doc() = "deep_vision_amd native input-pipeline runtime (TFRecord IO, Example decoding, batch collation)";
  m.def("crc32c", [](py::bytes b) { std::string s = b; return crc32c((const uint8_t*)s.data(), s.size()); });
  m.def("masked_crc32c", [](py::bytes b) { std::string s = b; return masked_crc((const uint8_t*)s.data(), s.size()); });
  py::class_<RecordWriter>(m, "RecordWriter")
      .def(py::init<const std::string&>())
      .def("write", &RecordWriter::write)
      .def("flush", &RecordWriter::flush)
      .def("close", &RecordWriter::close);
  py::class_<RecordReader>(m, "RecordReader")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("check_crc") = true)
      .def("next", &RecordReader::next)
      .def("read_at", &RecordReader::read_at)
      .def("reset", &RecordReader::reset);
  m.def("index_file", &index_file);
  m.def("parse_example", &parse_example);
  m.def("normalize_batch", &normalize_batch, py::arg("src"), py::arg("dst"), py::arg("mean"), py::arg("std"),
        py::arg("scale") = 255.f, py::arg("threads") = 8);
}
