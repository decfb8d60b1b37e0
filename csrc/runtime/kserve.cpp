// See kserve.h.
#include "kserve.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace arena {

namespace {

// ---------------------------------------------------------------- minimal JSON scanning
size_t skip_ws(const std::string& s, size_t i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  return i;
}

// s[i] == '"': the decoded string and the index past the closing quote (npos on a malformed string)
size_t scan_string(const std::string& s, size_t i, std::string* out) {
  if (i >= s.size() || s[i] != '"') return std::string::npos;
  ++i;
  while (i < s.size()) {
    const char c = s[i];
    if (c == '"') return i + 1;
    if (c == '\\') {
      if (i + 1 >= s.size()) return std::string::npos;
      const char e = s[i + 1];
      if (out) {
        switch (e) {
          case 'n': out->push_back('\n'); break;
          case 't': out->push_back('\t'); break;
          case 'r': out->push_back('\r'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'u': out->push_back('?'); break;  // names here are ASCII; a \u escape is kept as a placeholder
          default: out->push_back(e);
        }
      }
      i += e == 'u' ? 6 : 2;
      continue;
    }
    if (out) out->push_back(c);
    ++i;
  }
  return std::string::npos;
}

// Nesting bound of skip_value: the KServe messages read here nest at most four levels (header -> inputs ->
// tensor -> parameters); a hostile header of ~1 MB of '[' would otherwise recurse once per byte and overflow an
// I/O thread's stack.
constexpr int kMaxJsonDepth = 32;

// index past the JSON value starting at s[i] (after whitespace), npos if malformed or nested deeper than
// kMaxJsonDepth
size_t skip_value(const std::string& s, size_t i, int depth = 0) {
  i = skip_ws(s, i);
  if (i >= s.size()) return std::string::npos;
  const char c = s[i];
  if (c == '"') return scan_string(s, i, nullptr);
  if (c == '{' || c == '[') {
    if (depth >= kMaxJsonDepth) return std::string::npos;
    const char close = c == '{' ? '}' : ']';
    ++i;
    i = skip_ws(s, i);
    if (i < s.size() && s[i] == close) return i + 1;
    while (i < s.size()) {
      if (c == '{') {
        i = scan_string(s, skip_ws(s, i), nullptr);
        if (i == std::string::npos) return i;
        i = skip_ws(s, i);
        if (i >= s.size() || s[i] != ':') return std::string::npos;
        ++i;
      }
      i = skip_value(s, i, depth + 1);
      if (i == std::string::npos) return i;
      i = skip_ws(s, i);
      if (i < s.size() && s[i] == ',') {
        ++i;
        continue;
      }
      if (i < s.size() && s[i] == close) return i + 1;
      return std::string::npos;
    }
    return std::string::npos;
  }
  while (i < s.size() && s[i] != ',' && s[i] != '}' && s[i] != ']' && s[i] != ' ' && s[i] != '\n' && s[i] != '\r' &&
         s[i] != '\t')
    ++i;
  return i;
}

// visit(key, value_begin, value_end) for every member of the object at s[i]; false if malformed
template <class F>
bool for_members(const std::string& s, size_t i, F&& visit) {
  i = skip_ws(s, i);
  if (i >= s.size() || s[i] != '{') return false;
  i = skip_ws(s, i + 1);
  if (i < s.size() && s[i] == '}') return true;
  while (i < s.size()) {
    std::string key;
    i = scan_string(s, skip_ws(s, i), &key);
    if (i == std::string::npos) return false;
    i = skip_ws(s, i);
    if (i >= s.size() || s[i] != ':') return false;
    const size_t v0 = skip_ws(s, i + 1), v1 = skip_value(s, v0);
    if (v1 == std::string::npos) return false;
    visit(key, v0, v1);
    i = skip_ws(s, v1);
    if (i < s.size() && s[i] == ',') {
      ++i;
      continue;
    }
    return i < s.size() && s[i] == '}';
  }
  return false;
}

// visit(value_begin, value_end) for every element of the array at s[i]
template <class F>
bool for_elements(const std::string& s, size_t i, F&& visit) {
  i = skip_ws(s, i);
  if (i >= s.size() || s[i] != '[') return false;
  i = skip_ws(s, i + 1);
  if (i < s.size() && s[i] == ']') return true;
  while (i < s.size()) {
    const size_t v0 = skip_ws(s, i), v1 = skip_value(s, v0);
    if (v1 == std::string::npos) return false;
    visit(v0, v1);
    i = skip_ws(s, v1);
    if (i < s.size() && s[i] == ',') {
      ++i;
      continue;
    }
    return i < s.size() && s[i] == ']';
  }
  return false;
}

int64_t as_int(const std::string& s, size_t a, size_t b) { return std::strtoll(s.substr(a, b - a).c_str(), nullptr, 10); }

struct TensorDesc {
  std::string name, datatype;
  std::vector<int64_t> shape;
  int64_t binary_size = -1;
};

// the "inputs" / "outputs" array of a KServe message header
bool parse_tensors(const std::string& hdr, const char* field, std::vector<TensorDesc>& out, std::string* id) {
  bool found = false, ok = true;
  const bool good = for_members(hdr, 0, [&](const std::string& key, size_t v0, size_t v1) {
    (void)v1;
    if (key == "id" && id != nullptr && hdr[v0] == '"') scan_string(hdr, v0, id);
    if (key != field) return;
    found = true;
    ok = for_elements(hdr, v0, [&](size_t e0, size_t) {
      TensorDesc t;
      for_members(hdr, e0, [&](const std::string& k, size_t a, size_t b) {
        if (k == "name") scan_string(hdr, a, &t.name);
        else if (k == "datatype") scan_string(hdr, a, &t.datatype);
        else if (k == "shape")
          for_elements(hdr, a, [&](size_t x0, size_t x1) { t.shape.push_back(as_int(hdr, x0, x1)); });
        else if (k == "parameters")
          for_members(hdr, a, [&](const std::string& pk, size_t p0, size_t p1) {
            if (pk == "binary_data_size") t.binary_size = as_int(hdr, p0, p1);
          });
        (void)b;
      });
      out.push_back(std::move(t));
    });
  });
  return good && found && ok;
}

void json_str(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char ch : s) {
    if (ch == '"' || ch == '\\') {
      out.push_back('\\');
      out.push_back((char)ch);
    } else if (ch < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", ch);
      out += b;
    } else {
      out.push_back((char)ch);
    }
  }
  out.push_back('"');
}

void json_f(std::string& out, double v) {
  if (!std::isfinite(v)) {
    out += "null";
    return;
  }
  char b[32];
  snprintf(b, sizeof b, "%.9g", v);
  out += b;
}

void put_u32(std::string& s, uint32_t v) {
  const char b[4] = {(char)(v & 0xff), (char)((v >> 8) & 0xff), (char)((v >> 16) & 0xff), (char)(v >> 24)};
  s.append(b, 4);
}

bool write_full(int fd, const char* p, size_t n) {
  while (n > 0) {
    const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

}  // namespace

// ---------------------------------------------------------------- server side
bool kserve_parse_bytes_input(const std::string& body, int64_t ihcl, const std::string& input, size_t& off,
                              size_t& len, std::string& err) {
  if (ihcl < 0) {
    err = "the " + input + " input must use the binary tensor data extension (Inference-Header-Content-Length)";
    return false;
  }
  if ((size_t)ihcl > body.size()) {
    err = "Inference-Header-Content-Length exceeds the request body";
    return false;
  }
  const std::string hdr = body.substr(0, (size_t)ihcl);
  std::vector<TensorDesc> ins;
  if (!parse_tensors(hdr, "inputs", ins, nullptr)) {
    err = "malformed inference request header";
    return false;
  }
  // every size is client data: bound each one by what is left of the body before it is added, so no sum can
  // wrap around (sizes near 2^63 would otherwise move `bin` in front of the buffer)
  size_t bin = (size_t)ihcl;
  for (const TensorDesc& t : ins) {
    if (t.binary_size < 0 && t.binary_size != -1) {
      err = "negative binary_data_size";
      return false;
    }
    if (t.binary_size > 0 && (uint64_t)t.binary_size > body.size() - bin) {
      err = t.name + ": binary_data_size exceeds the request body";
      return false;
    }
    if (t.name != input) {
      if (t.binary_size > 0) bin += (size_t)t.binary_size;
      continue;
    }
    if (t.datatype != "BYTES") {
      err = input + " must be BYTES";
      return false;
    }
    if (t.binary_size < 4) {
      err = input + ": missing or inconsistent binary_data_size";
      return false;
    }
    int64_t n = 1;
    for (int64_t d : t.shape) {
      if (d < 0 || d > 1) {
        n = -1;
        break;
      }
      n *= d;
    }
    if (n != 1) {
      err = input + " must hold exactly one encoded image";
      return false;
    }
    const unsigned char* p = (const unsigned char*)body.data() + bin;
    const uint32_t l = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    if ((uint64_t)l + 4 > (uint64_t)t.binary_size) {
      err = input + ": element length exceeds its binary data";
      return false;
    }
    off = bin + 4;
    len = l;
    return true;
  }
  err = "expected input " + input;
  return false;
}

std::string kserve_build_response(const std::string& model, const std::string& id, const RequestResult& r,
                                  bool binary, int64_t* ihcl) {
  const int n = (int)r.det.size();
  std::vector<float> det((size_t)n * 6), logits((size_t)n * 5), probs((size_t)n * 5);
  std::vector<int32_t> ids((size_t)n * 5);
  for (int i = 0; i < n; ++i) {
    const Detection& d = r.det[i];
    const float row[6] = {d.x1, d.y1, d.x2, d.y2, d.conf, (float)d.cls};
    std::memcpy(&det[(size_t)i * 6], row, sizeof row);
    for (int k = 0; k < 5; ++k) {
      const bool have = i < (int)r.topk.size();
      ids[(size_t)i * 5 + k] = have ? r.topk[i].idx[k] : -1;
      logits[(size_t)i * 5 + k] = have ? r.topk[i].logit[k] : 0.f;
      probs[(size_t)i * 5 + k] = have ? r.topk[i].prob[k] : 0.f;
    }
  }
  const float stage[4] = {(float)std::max(0.0, r.det_ms), (float)std::max(0.0, r.cls_ms), (float)(r.queue_us / 1e3),
                          (float)(r.compute_us / 1e3)};
  struct Out {
    const char* name;
    const char* dtype;
    std::vector<int64_t> shape;
    const void* data;
    size_t bytes;
    bool is_int;
  };
  const Out outs[] = {
      {"DETECTIONS", "FP32", {n, 6}, det.data(), det.size() * 4, false},
      {"CLASS_IDS", "INT32", {n, 5}, ids.data(), ids.size() * 4, true},
      {"CLASS_LOGITS", "FP32", {n, 5}, logits.data(), logits.size() * 4, false},
      {"CLASS_PROBS", "FP32", {n, 5}, probs.data(), probs.size() * 4, false},
      {"STAGE_MS", "FP32", {4}, stage, sizeof stage, false},
  };
  std::string h = "{\"model_name\":";
  json_str(h, model);
  h += ",\"model_version\":\"1\"";
  if (!id.empty()) {
    h += ",\"id\":";
    json_str(h, id);
  }
  h += ",\"outputs\":[";
  bool first = true;
  for (const Out& o : outs) {
    if (!first) h += ',';
    first = false;
    h += "{\"name\":\"";
    h += o.name;
    h += "\",\"datatype\":\"";
    h += o.dtype;
    h += "\",\"shape\":[";
    for (size_t k = 0; k < o.shape.size(); ++k) h += (k ? "," : "") + std::to_string(o.shape[k]);
    h += "]";
    if (binary) {
      h += ",\"parameters\":{\"binary_data_size\":" + std::to_string(o.bytes) + "}}";
    } else {
      h += ",\"data\":[";
      const size_t cnt = o.bytes / 4;
      for (size_t k = 0; k < cnt; ++k) {
        if (k) h += ',';
        if (o.is_int) h += std::to_string(((const int32_t*)o.data)[k]);
        else json_f(h, ((const float*)o.data)[k]);
      }
      h += "]}";
    }
  }
  h += "]}";
  if (!binary) {
    *ihcl = -1;
    return h;
  }
  *ihcl = (int64_t)h.size();
  for (const Out& o : outs) h.append((const char*)o.data, o.bytes);
  return h;
}

std::string kserve_model_metadata(const std::string& model) {
  std::string s = "{\"name\":";
  json_str(s, model);
  s += ",\"versions\":[\"1\"],\"platform\":\"ensemble\",\"inputs\":[{\"name\":\"IMAGE_BYTES\",\"datatype\":\"BYTES\","
       "\"shape\":[1]}],\"outputs\":[{\"name\":\"DETECTIONS\",\"datatype\":\"FP32\",\"shape\":[-1,6]},"
       "{\"name\":\"CLASS_IDS\",\"datatype\":\"INT32\",\"shape\":[-1,5]},{\"name\":\"CLASS_LOGITS\",\"datatype\":"
       "\"FP32\",\"shape\":[-1,5]},{\"name\":\"CLASS_PROBS\",\"datatype\":\"FP32\",\"shape\":[-1,5]},"
       "{\"name\":\"STAGE_MS\",\"datatype\":\"FP32\",\"shape\":[4]}]}";
  return s;
}

// ---------------------------------------------------------------- client side
std::string kserve_build_request(const std::string& upload, const std::string& id, int64_t* ihcl) {
  std::string h = "{";
  if (!id.empty()) {
    h += "\"id\":";
    json_str(h, id);
    h += ',';
  }
  h += "\"inputs\":[{\"name\":\"IMAGE_BYTES\",\"shape\":[1],\"datatype\":\"BYTES\",\"parameters\":"
       "{\"binary_data_size\":" +
       std::to_string(upload.size() + 4) + "}}],\"outputs\":[";
  const char* outs[] = {"DETECTIONS", "CLASS_IDS", "CLASS_LOGITS", "CLASS_PROBS", "STAGE_MS"};
  for (int i = 0; i < 5; ++i) {
    if (i) h += ',';
    h += "{\"name\":\"";
    h += outs[i];
    h += "\",\"parameters\":{\"binary_data\":true}}";
  }
  h += "]}";
  *ihcl = (int64_t)h.size();
  put_u32(h, (uint32_t)upload.size());
  h += upload;
  return h;
}

bool kserve_parse_response(const std::string& body, int64_t ihcl, RequestResult& r, std::string& err) {
  if (ihcl < 0 || (size_t)ihcl > body.size()) {
    err = "model server answer without binary outputs";
    return false;
  }
  const std::string hdr = body.substr(0, (size_t)ihcl);
  std::vector<TensorDesc> outs;
  if (!parse_tensors(hdr, "outputs", outs, nullptr)) {
    err = "malformed inference response header";
    return false;
  }
  size_t pos = (size_t)ihcl;
  const float *det = nullptr, *logit = nullptr, *prob = nullptr, *stage = nullptr;
  const int32_t* ids = nullptr;
  int64_t n = -1, n_ids = -1, n_logit = -1, n_prob = -1;
  // element count of a shape with every dimension checked (non-negative, product bounded by the body size), -1 if
  // the shape is unusable
  auto count = [&](const std::vector<int64_t>& shape) -> int64_t {
    uint64_t c = 1;
    for (int64_t d : shape) {
      if (d < 0) return -1;
      if (d != 0 && c > (uint64_t)body.size() / (uint64_t)d) return -1;
      c *= (uint64_t)d;
    }
    return (int64_t)c;
  };
  // rows of an [n, cols] output, -1 when the shape is not that
  auto rows = [](const std::vector<int64_t>& shape, int64_t cols) -> int64_t {
    return shape.size() == 2 && shape[1] == cols && shape[0] >= 0 ? shape[0] : -1;
  };
  for (const TensorDesc& t : outs) {
    if (t.binary_size < 0 || (uint64_t)t.binary_size > body.size() - pos) {
      err = "output " + t.name + ": missing or inconsistent binary_data_size";
      return false;
    }
    const void* p = body.data() + pos;
    const int64_t cnt = count(t.shape);
    if (cnt < 0 || (uint64_t)cnt > (uint64_t)t.binary_size / 4 || cnt * 4 != t.binary_size) {
      err = "output " + t.name + ": shape and binary size disagree";
      return false;
    }
    if (t.name == "DETECTIONS") {
      det = (const float*)p;
      n = rows(t.shape, 6);
    } else if (t.name == "CLASS_IDS") {
      ids = (const int32_t*)p;
      n_ids = rows(t.shape, 5);
    } else if (t.name == "CLASS_LOGITS") {
      logit = (const float*)p;
      n_logit = rows(t.shape, 5);
    } else if (t.name == "CLASS_PROBS") {
      prob = (const float*)p;
      n_prob = rows(t.shape, 5);
    } else if (t.name == "STAGE_MS" && cnt >= 4) {
      stage = (const float*)p;
    }
    pos += (size_t)t.binary_size;
  }
  if (det == nullptr || n < 0) {
    err = "answer without DETECTIONS [n, 6]";
    return false;
  }
  const bool have_cls = ids != nullptr || logit != nullptr || prob != nullptr;
  if (have_cls && (n_ids != n || n_logit != n || n_prob != n)) {
    err = "CLASS_IDS / CLASS_LOGITS / CLASS_PROBS must all be [n, 5] with n the DETECTIONS rows";
    return false;
  }
  r.det.resize((size_t)n);
  r.topk.assign(ids && logit && prob ? (size_t)n : 0, TopkResult{});
  r.det_count = (int)n;
  for (int64_t i = 0; i < n; ++i) {
    float row[6];
    std::memcpy(row, det + i * 6, sizeof row);  // the blob is unaligned inside the body
    Detection& d = r.det[(size_t)i];
    d.x1 = row[0];
    d.y1 = row[1];
    d.x2 = row[2];
    d.y2 = row[3];
    d.conf = row[4];
    d.cls = (int)row[5];
    if (!r.topk.empty()) {
      TopkResult& t = r.topk[(size_t)i];
      std::memcpy(t.idx, ids + i * 5, 5 * sizeof(int32_t));
      std::memcpy(t.logit, logit + i * 5, 5 * sizeof(float));
      std::memcpy(t.prob, prob + i * 5, 5 * sizeof(float));
    }
  }
  if (stage != nullptr) {
    float st[4];
    std::memcpy(st, stage, sizeof st);
    r.det_ms = st[0];
    r.cls_ms = st[1];
    r.queue_us = st[2] * 1e3;
    r.compute_us = st[3] * 1e3;
  }
  return true;
}

KServeProxy::KServeProxy(std::string host, int port, std::string model, int conns, int timeout_ms)
    : KServeProxy(std::vector<KServeUpstream>{KServeUpstream{std::move(host), port}}, std::move(model), conns,
                  timeout_ms) {}

KServeProxy::KServeProxy(std::vector<KServeUpstream> ups, std::string model, int conns, int timeout_ms)
    : model_(std::move(model)), timeout_ms_(timeout_ms) {
  if (ups.empty()) throw std::runtime_error("KServeProxy: no upstream");
  for (auto& u : ups) {
    ups_.emplace_back();
    ups_.back().host = u.host;
    ups_.back().port = u.port;
  }
  for (int i = 0; i < std::max(1, conns); ++i) threads_.emplace_back([this, i] { worker(i); });
}

int KServeProxy::pick(int rotation) const {
  const int n = (int)ups_.size();
  int best = rotation % n, best_load = ups_[(size_t)best].inflight.load(std::memory_order_relaxed);
  for (int k = 1; k < n && best_load > 0; ++k) {
    const int u = (rotation + k) % n;
    const int l = ups_[(size_t)u].inflight.load(std::memory_order_relaxed);
    if (l < best_load) {
      best = u;
      best_load = l;
    }
  }
  return best;
}

KServeProxy::~KServeProxy() { stop(); }

void KServeProxy::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ && threads_.empty()) return;
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  std::deque<Task> left;
  {
    std::lock_guard<std::mutex> lk(mu_);
    left.swap(q_);
  }
  for (auto& t : left) {
    ProxyReply r;
    r.error = "gateway stopping";
    t.done(std::move(r));
  }
}

void KServeProxy::submit(std::string upload, std::function<void(ProxyReply&&)> done) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!stop_) {
      q_.push_back(Task{std::move(upload), std::move(done)});
      cv_.notify_one();
      return;
    }
  }
  ProxyReply r;
  r.error = "gateway stopping";
  done(std::move(r));
}

int KServeProxy::connect_upstream(int u, std::string& err) const {
  const std::string& host = ups_[(size_t)u].host;
  const int port = ups_[(size_t)u].port;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  if (rc != 0 || res == nullptr) {
    err = std::string("cannot resolve model server host ") + host + ": " + gai_strerror(rc);
    return -1;
  }
  const int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0 || ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    err = "cannot connect to the model server at " + host + ":" + std::to_string(port) + ": " + strerror(errno);
    if (fd >= 0) ::close(fd);
    freeaddrinfo(res);
    return -1;
  }
  freeaddrinfo(res);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  return fd;
}

bool KServeProxy::roundtrip(int& fd, const std::string& req, int& status, int64_t& ihcl, std::string& body,
                            std::string& err, RoundtripFail* fail) {
  RoundtripFail dummy;
  RoundtripFail& f = fail != nullptr ? *fail : dummy;
  f = RoundtripFail::None;
  if (!write_full(fd, req.data(), req.size())) {
    err = "send to the model server failed";
    f = RoundtripFail::Send;
    return false;
  }
  std::string in;
  size_t hend = std::string::npos;
  int64_t clen = -1;
  ihcl = -1;
  char buf[65536];
  while (true) {
    if (hend == std::string::npos) {
      hend = in.find("\r\n\r\n");
      if (hend != std::string::npos) {
        const size_t le = in.find("\r\n");
        const std::string line = in.substr(0, le);
        const size_t sp = line.find(' ');
        status = sp == std::string::npos ? 0 : std::atoi(line.c_str() + sp + 1);
        size_t p = le + 2;
        while (p < hend) {
          size_t e = in.find("\r\n", p);
          if (e == std::string::npos || e > hend) e = hend;
          const std::string h = in.substr(p, e - p);
          const size_t colon = h.find(':');
          if (colon != std::string::npos) {
            std::string name = h.substr(0, colon);
            for (auto& ch : name) ch = (char)std::tolower((unsigned char)ch);
            const long long v = std::atoll(h.c_str() + colon + 1);
            if (name == "content-length") clen = v;
            else if (name == "inference-header-content-length") ihcl = v;
          }
          p = e + 2;
        }
        if (clen < 0) {
          err = "model server answer without Content-Length";
          f = RoundtripFail::Protocol;
          return false;
        }
      }
    }
    if (hend != std::string::npos && in.size() >= hend + 4 + (size_t)clen) break;
    pollfd pf{fd, POLLIN, 0};
    const int pr = ::poll(&pf, 1, timeout_ms_);
    if (pr <= 0) {
      if (pr < 0 && errno == EINTR) continue;
      err = pr == 0 ? "model server timed out" : "poll failed";
      f = pr == 0 ? RoundtripFail::Timeout : RoundtripFail::Protocol;
      return false;
    }
    const ssize_t r = ::recv(fd, buf, sizeof buf, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      err = "model server closed the connection";
      // a keep-alive connection the server closed before answering anything: safe to resend on a new one
      f = in.empty() ? RoundtripFail::ClosedEarly : RoundtripFail::Protocol;
      return false;
    }
    in.append(buf, (size_t)r);
  }
  body.assign(in, hend + 4, (size_t)clen);
  return true;
}

bool KServeProxy::upstream_ready() {
  for (int u = 0; u < (int)ups_.size(); ++u) {
    std::string err;
    int fd = connect_upstream(u, err);
    if (fd < 0) return false;
    const std::string req =
        "GET /v2/health/ready HTTP/1.1\r\nHost: " + ups_[(size_t)u].host + "\r\nContent-Length: 0\r\n\r\n";
    int status = 0;
    int64_t ihcl = -1;
    std::string body;
    const bool ok = roundtrip(fd, req, status, ihcl, body, err) && status == 200;
    ::close(fd);
    if (!ok) return false;
  }
  return true;
}

void KServeProxy::worker(int index) {
  pthread_setname_np(pthread_self(), "arena-kproxy");
  std::vector<int> fds(ups_.size(), -1);
  uint64_t seq = 0;
  int rotation = index;
  std::string req;
  while (true) {
    Task t;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) break;  // stopping
      t = std::move(q_.front());
      q_.pop_front();
    }
    const int u = pick(rotation++);
    Up& up = ups_[(size_t)u];
    up.inflight.fetch_add(1, std::memory_order_relaxed);
    int& fd = fds[(size_t)u];
    ProxyReply rep;
    int64_t ihcl = -1;
    const std::string payload = kserve_build_request(t.upload, "", &ihcl);
    if (recycle_) recycle_->put(std::move(t.upload));
    req.clear();  // the worker's request buffer, reused
    req += "POST /v2/models/" + model_ + "/infer HTTP/1.1\r\nHost: " + up.host +
           "\r\nContent-Type: application/octet-stream\r\nInference-Header-Content-Length: " +
           std::to_string(ihcl) + "\r\nContent-Length: " + std::to_string(payload.size()) + "\r\n\r\n";
    req += payload;
    std::string body, err;
    bool ok = false;
    for (int attempt = 0; attempt < 2 && !ok; ++attempt) {
      if (fd < 0) {
        fd = connect_upstream(u, err);
        if (fd < 0) break;
        if (seq++ > 0) ++reconnects_;
      }
      int64_t rihcl = -1;
      RoundtripFail why = RoundtripFail::None;
      ok = roundtrip(fd, req, rep.status, rihcl, body, err, &why);
      if (!ok) {
        ::close(fd);
        fd = -1;
        // resend only what the model server cannot have started: a failed send or a keep-alive connection closed
        // before any answer byte.  A timeout means an overloaded server: answer 504 rather than doubling its load.
        if (why == RoundtripFail::Timeout) {
          rep.status = 504;
          break;
        }
        if (why != RoundtripFail::Send && why != RoundtripFail::ClosedEarly) break;
        continue;
      }
      if (rep.status == 200) {
        if (!kserve_parse_response(body, rihcl, rep.result, err)) rep.error = err;
      } else {
        rep.error = body.empty() ? "model server error " + std::to_string(rep.status) : body;
      }
    }
    if (!ok) {
      rep.error = err.empty() ? "model server unreachable" : err;
      if (rep.status == 200) rep.status = 0;
    }
    up.inflight.fetch_sub(1, std::memory_order_relaxed);
    up.forwarded.fetch_add(1, std::memory_order_relaxed);
    ++forwarded_;
    t.done(std::move(rep));
  }
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
}

}  // namespace arena
