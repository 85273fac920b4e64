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
// The logic lives in io_core.h (pure C++, sanitizer-tested by io_selftest.cpp); this file is the
// pybind11 glue. The GIL is released around file IO and the pixel loop.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "io_core.h"

namespace py = pybind11;

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
    uint8_t hdr[12];
    dvio::frame_header(s.size(), hdr);
    const uint32_t dc = dvio::masked_crc((const uint8_t*)s.data(), s.size());
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
      ok = dvio::read_record(f_, out, check_, path_);
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
      ok = dvio::read_record(f_, out, check_, path_);
    }
    if (!ok) throw std::runtime_error("no record at offset " + std::to_string(offset) + " in " + path_);
    return py::bytes(out);
  }
  void reset() { fseeko(f_, 0, SEEK_SET); }

 private:
  std::string path_;
  bool check_;
  FILE* f_ = nullptr;
};

static py::object feature_to_py(const dvio::Feature& f) {
  switch (f.kind) {
    case dvio::Kind::Bytes: {
      py::list out;
      for (const auto& s : f.bytes) out.append(py::bytes(s));
      return py::make_tuple("bytes", out);
    }
    case dvio::Kind::Float: return py::make_tuple("float", py::cast(f.floats));
    case dvio::Kind::Int64: return py::make_tuple("int64", py::cast(f.ints));
    default: return py::make_tuple("empty", py::list());
  }
}

static py::dict parse_example(py::bytes data) {
  std::string s = data;
  auto feats = dvio::parse_example((const uint8_t*)s.data(), s.size());
  py::dict out;
  for (const auto& kv : feats) out[py::str(kv.first)] = feature_to_py(kv.second);
  return out;
}

static void normalize_batch(py::array_t<uint8_t, py::array::c_style> src, py::array_t<float, py::array::c_style> dst,
                            std::vector<float> mean, std::vector<float> stdv, float scale, int threads) {
  if (src.ndim() != 4 || dst.ndim() != 4) throw std::runtime_error("normalize_batch: 4-D arrays expected");
  const int64_t N = src.shape(0), H = src.shape(1), W = src.shape(2), C = src.shape(3);
  if (dst.shape(0) != N || dst.shape(1) != C || dst.shape(2) != H || dst.shape(3) != W)
    throw std::runtime_error("normalize_batch: dst must be (N, C, H, W)");
  const uint8_t* s = src.data();
  float* d = dst.mutable_data();
  py::gil_scoped_release nogil;
  dvio::normalize_batch(s, d, N, H, W, C, mean, stdv, scale, threads);
}

// (H, W, C) uint8 -> the (ch, cw, C) crop of its bilinear rescale to (outH, outW), GIL released.
// ``src`` may be a strided view with unit channel stride (e.g. the RGB channels of a decoder's
// RGBX buffer, exported without a copy: data/datasets.py load_rgb).
static py::array_t<uint8_t> resize_crop(py::array_t<uint8_t, py::array::forcecast> src, int64_t outH, int64_t outW,
                                        int64_t cy, int64_t cx, int64_t ch, int64_t cw) {
  if (src.ndim() != 3) throw std::runtime_error("resize_crop: expected an HWC array");
  const int64_t H = src.shape(0), W = src.shape(1), C = src.shape(2);
  if (src.strides(2) != 1 || src.strides(1) < C || src.strides(0) < W * src.strides(1))  // e.g. a flipped view
    src = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(src);
  const int64_t ps = src.strides(1), rs = src.strides(0);
  py::array_t<uint8_t> out({ch, cw, C});
  const uint8_t* s = src.data();
  uint8_t* d = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    dvio::resize_crop_bilinear(s, H, W, C, outH, outW, cy, cx, ch, cw, d, ps, rs);
  }
  return out;
}

static void color_jitter(py::array_t<uint8_t, py::array::c_style> img, std::vector<float> f, std::vector<int> order) {
  if (img.ndim() != 3 || img.shape(2) != 3 || f.size() != 3 || order.size() != 3)
    throw std::runtime_error("color_jitter: expected an HWC RGB uint8 array, 3 factors and an order");
  uint8_t* p = img.mutable_data();
  const int64_t n = img.shape(0) * img.shape(1);
  py::gil_scoped_release nogil;
  dvio::color_jitter(p, n, f.data(), order.data());
}

PYBIND11_MODULE(_io, m) {
  m.doc() = "deep_vision_amd native input-pipeline runtime (TFRecord IO, Example decoding, batch collation)";
  m.def("crc32c", [](py::bytes b) { std::string s = b; return dvio::crc32c((const uint8_t*)s.data(), s.size()); });
  m.def("masked_crc32c", [](py::bytes b) { std::string s = b; return dvio::masked_crc((const uint8_t*)s.data(), s.size()); });
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
  m.def("index_file", &dvio::index_file);
  m.def("parse_example", &parse_example);
  m.def("resize_crop", &resize_crop, py::arg("src"), py::arg("out_h"), py::arg("out_w"), py::arg("cy"), py::arg("cx"),
        py::arg("ch"), py::arg("cw"));
  m.def("color_jitter", &color_jitter, py::arg("img"), py::arg("factors"), py::arg("order"));
  m.def("normalize_batch", &normalize_batch, py::arg("src"), py::arg("dst"), py::arg("mean"), py::arg("std"),
        py::arg("scale") = 255.f, py::arg("threads") = 8);
}
