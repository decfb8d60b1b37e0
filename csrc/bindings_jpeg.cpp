// pybind11 bindings of the split JPEG decoder (runtime/jpeg_decode.h, kernels/jpeg_idct.hip): the host
// entropy decoder and reference reconstruction for tests / host-only decoding, and a stand-alone device
// reconstruction of a list of uploads (the kernel-vs-reference tests; the serving path runs the same kernels
// inside Executor::submit).
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/jpeg_desc.h"
#include "kernels/launch.h"
#include "runtime/jpeg_decode.h"

namespace py = pybind11;

namespace arena {

namespace {

const char* status_name(JpegStatus s) {
  return s == JpegStatus::Ok ? "ok" : (s == JpegStatus::Unsupported ? "unsupported" : "corrupt");
}

py::dict info_dict(const JpegInfo& in) {
  py::dict d;
  d["width"] = in.width;
  d["height"] = in.height;
  d["ncomp"] = in.ncomp;
  d["layout"] = in.layout;
  d["mcux"] = in.mcux;
  d["mcuy"] = in.mcuy;
  d["restart_interval"] = in.restart_interval;
  d["coef_count"] = in.coef_count;
  py::list comps;
  for (int c = 0; c < in.ncomp; ++c) {
    const JpegCompDesc& k = in.comp[c];
    py::dict e;
    e["h"] = k.h;
    e["v"] = k.v;
    e["bw"] = k.bw;
    e["bh"] = k.bh;
    e["cw"] = k.cw;
    e["ch"] = k.ch;
    e["coef_off"] = k.coef_off;
    comps.append(e);
  }
  d["comps"] = comps;
  return d;
}

struct Parsed {
  JpegInfo info;
  std::vector<int16_t> coef;
};

JpegStatus parse_decode(const std::string& data, Parsed& p, std::string& err, int64_t max_pixels) {
  const uint8_t* b = (const uint8_t*)data.data();
  JpegStatus st = jpeg_parse(b, data.size(), p.info, err, max_pixels);
  if (st != JpegStatus::Ok) return st;
  p.coef.assign((size_t)p.info.coef_count, 0);
  return jpeg_decode_coefs(b, data.size(), p.info, p.coef.data(), err);
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " (" + what + ")");
}

int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

}  // namespace

void bind_jpeg(py::module& m) {
  m.attr("SIZEOF_JPEG_DESC") = (int)sizeof(JpegDesc);

  m.def(
      "jpeg_coefs",
      [](py::bytes data, int64_t max_pixels) {
        std::string s = data;
        Parsed p;
        std::string err;
        JpegStatus st;
        {
          py::gil_scoped_release nogil;
          st = parse_decode(s, p, err, max_pixels);
        }
        py::dict out = info_dict(p.info);
        out["status"] = status_name(st);
        out["error"] = err;
        py::array_t<int16_t> a((py::ssize_t)p.coef.size());
        if (!p.coef.empty()) std::memcpy(a.mutable_data(), p.coef.data(), p.coef.size() * sizeof(int16_t));
        out["coef"] = a;
        return out;
      },
      py::arg("data"), py::arg("max_pixels") = 0,
      "Host entropy decode: dict(status, error, geometry, comps, coef=int16 natural-order blocks).");

  m.def(
      "jpeg_decode_host",
      [](py::bytes data, int64_t max_pixels) -> py::object {
        std::string s = data;
        Parsed p;
        std::string err;
        JpegStatus st;
        std::vector<uint8_t> rgb;
        {
          py::gil_scoped_release nogil;
          st = parse_decode(s, p, err, max_pixels);
          if (st == JpegStatus::Ok) {
            rgb.resize((size_t)p.info.width * p.info.height * 3);
            jpeg_coefs_to_rgb(p.info, p.coef.data(), rgb.data());
          }
        }
        if (st != JpegStatus::Ok) return py::make_tuple(status_name(st), err, py::none());
        py::array_t<uint8_t> a({(py::ssize_t)p.info.height, (py::ssize_t)p.info.width, (py::ssize_t)3});
        std::memcpy(a.mutable_data(), rgb.data(), rgb.size());
        return py::make_tuple("ok", std::string(), a);
      },
      py::arg("data"), py::arg("max_pixels") = 0,
      "Whole decode on the host with the device kernels' arithmetic: (status, error, HxWx3 uint8 or None).");

  m.def(
      "jpeg_decode_device",
      [](std::vector<py::bytes> uploads, int device) {
        const int n = (int)uploads.size();
        std::vector<Parsed> ps(n);
        std::vector<JpegDesc> descs(n);
        int64_t off = 0, max_blocks = 0, max_pix = 0;
        std::vector<int64_t> coef_base(n), rgb_off(n);
        for (int i = 0; i < n; ++i) {
          std::string err;
          const std::string s = uploads[i];
          if (parse_decode(s, ps[i], err, 0) != JpegStatus::Ok) throw std::invalid_argument("upload " + std::to_string(i) + ": " + err);
          const JpegInfo& in = ps[i].info;
          rgb_off[i] = off;
          off = align256(off + (int64_t)in.width * in.height * 3);
          coef_base[i] = off;
          off = align256(off + in.coef_count * 2);
          descs[i] = jpeg_device_desc(in, coef_base[i], off, rgb_off[i]);
          off = align256(off + in.plane_bytes);
          max_blocks = std::max<int64_t>(max_blocks, descs[i].total_blocks);
          max_pix = std::max<int64_t>(max_pix, (int64_t)in.width * in.height);
        }
        py::list out;
        if (n == 0) return out;
        check(hipSetDevice(device), "hipSetDevice");
        uint8_t* pool = nullptr;
        JpegDesc* dd = nullptr;
        check(hipMalloc(&pool, (size_t)off), "hipMalloc pool");
        check(hipMalloc(&dd, sizeof(JpegDesc) * n), "hipMalloc descs");
        std::vector<std::vector<uint8_t>> rgb(n);
        try {
          check(hipMemset(pool, 0xCD, (size_t)off), "hipMemset");
          for (int i = 0; i < n; ++i)
            check(hipMemcpy(pool + coef_base[i], ps[i].coef.data(), ps[i].coef.size() * 2, hipMemcpyHostToDevice), "H2D coef");
          check(hipMemcpy(dd, descs.data(), sizeof(JpegDesc) * n, hipMemcpyHostToDevice), "H2D desc");
          jpeg_reconstruct(dd, pool, n, (int)max_blocks, max_pix, nullptr);
          check(hipGetLastError(), "jpeg_reconstruct launch");
          check(hipDeviceSynchronize(), "jpeg_reconstruct");
          for (int i = 0; i < n; ++i) {
            rgb[i].resize((size_t)ps[i].info.width * ps[i].info.height * 3);
            check(hipMemcpy(rgb[i].data(), pool + rgb_off[i], rgb[i].size(), hipMemcpyDeviceToHost), "D2H rgb");
          }
        } catch (...) {
          hipFree(pool);
          hipFree(dd);
          throw;
        }
        hipFree(pool);
        hipFree(dd);
        for (int i = 0; i < n; ++i) {
          py::array_t<uint8_t> a({(py::ssize_t)ps[i].info.height, (py::ssize_t)ps[i].info.width, (py::ssize_t)3});
          std::memcpy(a.mutable_data(), rgb[i].data(), rgb[i].size());
          out.append(a);
        }
        return out;
      },
      py::arg("uploads"), py::arg("device") = 0,
      "Entropy-decode on the host, reconstruct on the GPU (jpeg_idct.hip): list of HxWx3 uint8.");
}

}  // namespace arena
