// Malformed-message driver for the KServe-v2 binary-tensor codec (csrc/runtime/kserve.cpp), built host-only under
// AddressSanitizer by tests/test_native_http.py.  Requests reach kserve_parse_bytes_input straight from the model
// server's public REST port, and the gateway's kserve_parse_response reads whatever the upstream answers, so no
// header may make either read outside the body.
//
//   kserve_fuzz [iterations]
//
// 1. fixed hostile headers: ~1 MB of '[' (stack depth), binary_data_size values that wrap a 64-bit sum, negative
//    sizes, shapes whose element count overflows, DETECTIONS / CLASS_* row counts that disagree: all rejected;
// 2. valid request / response round trips parse to what was encoded;
// 3. random byte flips, truncations and digit rewrites of valid messages: any verdict, no memory error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "runtime/kserve.h"

namespace {

int failures = 0;

void expect(bool cond, const char* what) {
  if (!cond) {
    std::printf("FAIL: %s\n", what);
    ++failures;
  }
}

bool parse_req(const std::string& body, int64_t ihcl, size_t* off = nullptr, size_t* len = nullptr) {
  size_t o = 0, l = 0;
  std::string err;
  const bool ok = arena::kserve_parse_bytes_input(body, ihcl, "IMAGE_BYTES", o, l, err);
  if (ok) {
    // the contract: the element lies inside the body
    if (o > body.size() || l > body.size() - o) {
      std::printf("FAIL: accepted element outside the body (off %zu len %zu size %zu)\n", o, l, body.size());
      ++failures;
    }
  }
  if (off) *off = o;
  if (len) *len = l;
  return ok;
}

std::string hdr_with(const std::string& inputs) { return "{\"inputs\":[" + inputs + "]}"; }

std::string le32(uint32_t v) {
  std::string s(4, '\0');
  for (int i = 0; i < 4; ++i) s[i] = (char)((v >> (8 * i)) & 0xff);
  return s;
}

arena::RequestResult sample_result(int n) {
  arena::RequestResult r;
  for (int i = 0; i < n; ++i) {
    arena::Detection d{};
    d.x1 = 1.f + i;
    d.y1 = 2.f;
    d.x2 = 30.f + i;
    d.y2 = 40.f;
    d.conf = 0.5f + 0.01f * i;
    d.cls = i;
    r.det.push_back(d);
    arena::TopkResult t{};
    for (int k = 0; k < 5; ++k) {
      t.idx[k] = 10 * i + k;
      t.logit[k] = 5.f - k;
      t.prob[k] = 0.2f;
    }
    r.topk.push_back(t);
  }
  r.det_ms = 1.0;
  r.cls_ms = 2.0;
  return r;
}

bool parse_resp(const std::string& body, int64_t ihcl, arena::RequestResult* out = nullptr) {
  arena::RequestResult r;
  std::string err;
  const bool ok = arena::kserve_parse_response(body, ihcl, r, err);
  if (out) *out = r;
  return ok;
}

// a response with hand-written output descriptors (shape text, binary size) and `payload` bytes of zeros
std::string resp_with(const std::string& outputs, size_t payload, int64_t* ihcl) {
  std::string h = "{\"outputs\":[" + outputs + "]}";
  *ihcl = (int64_t)h.size();
  return h + std::string(payload, '\0');
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const std::string jpeg = "\xff\xd8 fake image bytes \xff\xd9";

  // ---- 1. requests: fixed hostile headers
  {
    const std::string deep(1 << 20, '[');
    const std::string body = "{\"inputs\":" + deep;
    expect(!parse_req(body, (int64_t)body.size()), "1 MB of '[' rejected");
    std::string deep_obj;
    for (int i = 0; i < 200000; ++i) deep_obj += "{\"a\":";
    const std::string body2 = "{\"inputs\":[{\"parameters\":" + deep_obj + "1}]}";
    expect(!parse_req(body2, (int64_t)body2.size()), "deeply nested objects rejected");
  }
  {
    // two other inputs whose sizes wrap the running offset to just under 2^64, then the image input
    const std::string h = hdr_with(
        "{\"name\":\"A\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":9223372036854775807}},"
        "{\"name\":\"B\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":9223372036854775800}},"
        "{\"name\":\"IMAGE_BYTES\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":30}}");
    const std::string body = h + le32((uint32_t)jpeg.size()) + jpeg;
    expect(!parse_req(body, (int64_t)h.size()), "wrapping binary_data_size sum rejected");
  }
  {
    const std::string h = hdr_with(
        "{\"name\":\"A\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":-5}},"
        "{\"name\":\"IMAGE_BYTES\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":30}}");
    const std::string body = h + le32((uint32_t)jpeg.size()) + jpeg;
    expect(!parse_req(body, (int64_t)h.size()), "negative binary_data_size rejected");
  }
  {
    const std::string h = hdr_with(
        "{\"name\":\"IMAGE_BYTES\",\"datatype\":\"BYTES\",\"shape\":[-1],\"parameters\":{\"binary_data_size\":" +
        std::to_string(jpeg.size() + 4) + "}}");
    const std::string body = h + le32((uint32_t)jpeg.size()) + jpeg;
    expect(!parse_req(body, (int64_t)h.size()), "negative shape rejected");
  }
  {
    // element length prefix larger than its binary data
    const std::string h = hdr_with(
        "{\"name\":\"IMAGE_BYTES\",\"datatype\":\"BYTES\",\"shape\":[1],\"parameters\":{\"binary_data_size\":" +
        std::to_string(jpeg.size() + 4) + "}}");
    const std::string body = h + le32(0xfffffff0u) + jpeg;
    expect(!parse_req(body, (int64_t)h.size()), "oversize element length rejected");
  }
  {
    // the valid request the gateway builds
    int64_t ihcl = -1;
    const std::string body = arena::kserve_build_request(jpeg, "rid", &ihcl);
    size_t off = 0, len = 0;
    expect(parse_req(body, ihcl, &off, &len), "valid request accepted");
    expect(len == jpeg.size() && body.compare(off, len, jpeg) == 0, "valid request element located");
  }

  // ---- 1b. responses: fixed hostile headers
  {
    int64_t ihcl = -1;
    const std::string body = arena::kserve_build_response("arena_pipeline", "", sample_result(3), true, &ihcl);
    arena::RequestResult r;
    expect(parse_resp(body, ihcl, &r), "valid response accepted");
    expect(r.det.size() == 3 && r.topk.size() == 3 && r.topk[2].idx[4] == 24 && r.det[1].cls == 1,
           "valid response decoded");
  }
  {
    int64_t ihcl = -1;  // DETECTIONS with 5 columns
    const std::string body = resp_with("{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[2,5],"
                                       "\"parameters\":{\"binary_data_size\":40}}",
                                       40, &ihcl);
    expect(!parse_resp(body, ihcl), "DETECTIONS [n,5] rejected");
  }
  {
    int64_t ihcl = -1;  // CLASS_IDS with fewer rows than DETECTIONS: the row loop would read past it
    const std::string body = resp_with(
        "{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[4,6],\"parameters\":{\"binary_data_size\":96}},"
        "{\"name\":\"CLASS_IDS\",\"datatype\":\"INT32\",\"shape\":[1,5],\"parameters\":{\"binary_data_size\":20}},"
        "{\"name\":\"CLASS_LOGITS\",\"datatype\":\"FP32\",\"shape\":[1,5],\"parameters\":{\"binary_data_size\":20}},"
        "{\"name\":\"CLASS_PROBS\",\"datatype\":\"FP32\",\"shape\":[1,5],\"parameters\":{\"binary_data_size\":20}}",
        156, &ihcl);
    expect(!parse_resp(body, ihcl), "CLASS_* rows disagreeing with DETECTIONS rejected");
  }
  {
    int64_t ihcl = -1;  // element count 2^62 * 4 overflows int64: must not pass the size check
    const std::string body = resp_with("{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[4611686018427387904,6],"
                                       "\"parameters\":{\"binary_data_size\":0}}",
                                       0, &ihcl);
    expect(!parse_resp(body, ihcl), "overflowing DETECTIONS shape rejected");
  }
  {
    int64_t ihcl = -1;
    const std::string body = resp_with("{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[-2,6],"
                                       "\"parameters\":{\"binary_data_size\":0}}",
                                       0, &ihcl);
    expect(!parse_resp(body, ihcl), "negative DETECTIONS rows rejected");
  }
  {
    int64_t ihcl = -1;
    const std::string body = resp_with("{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[1,6],"
                                       "\"parameters\":{\"binary_data_size\":18446744073709551600}}",
                                       24, &ihcl);
    expect(!parse_resp(body, ihcl), "huge output binary_data_size rejected");
  }

  // ---- 2./3. random mutations of valid messages
  std::mt19937 rng(1234);
  int64_t q_ihcl = -1, r_ihcl = -1;
  const std::string req = arena::kserve_build_request(jpeg, "id-1", &q_ihcl);
  const std::string resp = arena::kserve_build_response("m", "", sample_result(4), true, &r_ihcl);
  for (int it = 0; it < iters; ++it) {
    const bool is_req = (it & 1) == 0;
    std::string m = is_req ? req : resp;
    int64_t ihcl = is_req ? q_ihcl : r_ihcl;
    const int edits = 1 + (int)(rng() % 4);
    for (int e = 0; e < edits; ++e) {
      const int kind = (int)(rng() % 5);
      if (m.empty()) break;
      const size_t pos = rng() % m.size();
      if (kind == 0) {
        m[pos] = (char)(rng() & 0xff);
      } else if (kind == 1) {
        m.resize(pos);
      } else if (kind == 2 && pos < (size_t)ihcl) {
        if (m[pos] >= '0' && m[pos] <= '9') m.insert(pos, std::string(1 + rng() % 18, (char)('0' + rng() % 10)));
      } else if (kind == 3 && pos < (size_t)ihcl) {
        m.insert(pos, std::string(1 + rng() % 64, (rng() & 1) ? '[' : '{'));
      } else {
        ihcl = (int64_t)(rng() % (m.size() + 8)) - 4;
      }
    }
    if (is_req) parse_req(m, ihcl);
    else parse_resp(m, ihcl);
  }
  if (failures) {
    std::printf("kserve_fuzz: %d failures\n", failures);
    return 1;
  }
  std::printf("kserve_fuzz: ok (%d mutations)\n", iters);
  return 0;
}
