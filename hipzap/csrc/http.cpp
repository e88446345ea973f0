// hipzap native HTTP/1.1 front end (serving layer, SURVEY.md §1 L5 / §3.6 "warm request").
//
// Measured problem (profiles/r2_http): behind werkzeug's threaded WSGI server a POST /predict
// costs ~1.2 ms of GIL-held Python per request -> ~800 req/s per process, while the GPU serves
// ~11k inf/s. This server keeps the Flask app as THE application (every route, every body
// format, the Zappa contract) and takes only the hot route natively:
//   POST /predict with one uint8 HWC image of the plan's shape, as JSON {"image_b64", "shape"
//   [, "model"]} or as an .npy body -> base64/npy decode -> the request executor
//   (csrc/executor.cpp: pinned input, hipGraph replay, wait) -> softmax + top-5 -> the same
//   JSON schema as the Flask route (hipzap/serve/app.py predict()).
// And, once the AWD-LSTM backend is loaded (hz_http_set_lm), the reference's own route:
//   GET /inference [?seed=<int>][&words=<int>] (no prompt: the reference's request,
//   /root/reference/main.py:105-112) -> the continuous-batching decode scheduler
//   (csrc/lmserve.cpp hz_lmb_submit, blocking) -> the reference's detokenizer over a vocabulary
//   table whose per-word JSON fragments, capitalised forms and spacing flags Python computed
//   (serve/native_http.py set_lm: byte-identical to the Flask route's body) -> JSON.
// Anything else (other routes, batches, other keys or dtypes, query flags) goes to a Python
// callback that runs the WSGI app and answers through hz_http_respond(). One thread per
// keep-alive connection, blocking I/O; the GIL is only taken on the fallback path.
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

using PyHandler = HzHttpPyHandler;

struct Fast {
  void* exec = nullptr;  // HzExecutor over the plan's contexts
  int H = 0, W = 0, C = 0;
  int out_floats = 0, classes = 0, probs = 0;
  std::string model;
};

// The GET /inference route: the decode scheduler and the detokenizer's vocabulary table.
struct Lm {
  void* sched = nullptr;     // csrc/lmserve.cpp scheduler
  int V = 0, maxn = 0, dflt = 200, empty_id = 0;
  std::vector<std::string> w, wc;  // JSON-escaped word / its capitalised form (no quotes)
  std::vector<uint8_t> fl;         // bit0 word in NO_SPACE, bit1 capitalised in NO_SPACE,
                                   // bit2 word in CAPITALIZE_AFTER, bit3 capitalised in CAPITALIZE_AFTER
};

struct Server {
  int lfd = -1;
  std::atomic<bool> stop{false};
  std::atomic<int> live{0};
  std::thread acceptor;
  PyHandler py = nullptr;
  Fast fast;
  std::atomic<bool> has_fast{false};
  std::mutex fast_mu;
  std::atomic<uint64_t> n_fast{0}, n_py{0}, n_bad{0};
  std::shared_ptr<const Lm> lm;  // (replaced whole under lm_mu; a request keeps its copy alive)
  std::mutex lm_mu;
};

struct PyReq {
  std::string out;
  bool keep = true;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool send_str(int fd, const std::string& s) { return send_all(fd, s.data(), s.size()); }

std::string simple(int code, const std::string& body, bool keep) {
  char h[256];
  snprintf(h, sizeof(h),
           "HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n"
           "Access-Control-Allow-Origin: *\r\nConnection: %s\r\n\r\n",
           code, reason(code), body.size(), keep ? "keep-alive" : "close");
  return std::string(h) + body;
}

// ---------------------------------------------------------------- small parsers
int b64val(unsigned char c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+' || c == '-') return 62;
  if (c == '/' || c == '_') return 63;
  return -1;
}

// decode exactly `want` bytes of standard base64 (padding optional); false on any other length
bool b64decode(const char* s, size_t n, uint8_t* out, size_t want) {
  while (n && (s[n - 1] == '=')) --n;
  if ((n * 3) / 4 != want) return false;
  size_t o = 0, i = 0;
  for (; i + 4 <= n; i += 4) {
    int a = b64val(s[i]), b = b64val(s[i + 1]), c = b64val(s[i + 2]), d = b64val(s[i + 3]);
    if ((a | b | c | d) < 0) return false;
    const unsigned v = (unsigned)a << 18 | (unsigned)b << 12 | (unsigned)c << 6 | (unsigned)d;
    out[o++] = (uint8_t)(v >> 16);
    out[o++] = (uint8_t)(v >> 8);
    out[o++] = (uint8_t)v;
  }
  const size_t rem = n - i;
  if (rem == 2 || rem == 3) {
    int a = b64val(s[i]), b = b64val(s[i + 1]), c = rem == 3 ? b64val(s[i + 2]) : 0;
    if ((a | b | c) < 0) return false;
    const unsigned v = (unsigned)a << 18 | (unsigned)b << 12 | (unsigned)c << 6;
    out[o++] = (uint8_t)(v >> 16);
    if (rem == 3) out[o++] = (uint8_t)(v >> 8);
  } else if (rem == 1) {
    return false;
  }
  return o == want;
}

void skip_ws(const char*& p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
}

// a JSON string without escapes (keys, base64, model names); false otherwise
bool json_str(const char*& p, const char* e, const char** s, size_t* n) {
  if (p >= e || *p != '"') return false;
  const char* q = ++p;
  while (p < e && *p != '"') {
    if (*p == '\\') return false;
    ++p;
  }
  if (p >= e) return false;
  *s = q;
  *n = (size_t)(p - q);
  ++p;
  return true;
}

bool json_int_array(const char*& p, const char* e, std::vector<long>& v) {
  if (p >= e || *p != '[') return false;
  ++p;
  for (;;) {
    skip_ws(p, e);
    if (p < e && *p == ']' && v.empty()) {
      ++p;
      return true;
    }
    // bounded decimal parse: never reads past e (strtol would run on into whatever follows the
    // body in the connection buffer)
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
    const char* d0 = p;
    long x = 0;
    while (p < e && *p >= '0' && *p <= '9') {
      if (x > 100000000L) return false;  // shapes are small; refuse instead of overflowing
      x = x * 10 + (*p++ - '0');
    }
    if (p == d0) return false;
    v.push_back(neg ? -x : x);
    skip_ws(p, e);
    if (p < e && *p == ',') {
      ++p;
      continue;
    }
    if (p < e && *p == ']') {
      ++p;
      return true;
    }
    return false;
  }
}

// {"image_b64": "...", "shape": [..], "model": "..."} and nothing else -> true
bool parse_json_image(const char* b, size_t n, const char** img, size_t* img_n, std::vector<long>& shape,
                      std::string& model) {
  const char *p = b, *e = b + n;
  skip_ws(p, e);
  if (p >= e || *p != '{') return false;
  ++p;
  bool have_img = false, have_shape = false;
  for (;;) {
    skip_ws(p, e);
    const char* k;
    size_t kn;
    if (!json_str(p, e, &k, &kn)) return false;
    skip_ws(p, e);
    if (p >= e || *p != ':') return false;
    ++p;
    skip_ws(p, e);
    if (kn == 9 && !memcmp(k, "image_b64", 9)) {
      if (!json_str(p, e, img, img_n)) return false;
      have_img = true;
    } else if (kn == 5 && !memcmp(k, "shape", 5)) {
      if (!json_int_array(p, e, shape)) return false;
      have_shape = true;
    } else if (kn == 5 && !memcmp(k, "model", 5)) {
      const char* m;
      size_t mn;
      if (!json_str(p, e, &m, &mn)) return false;
      model.assign(m, mn);
    } else {
      return false;  // any other key: the Flask route decides
    }
    skip_ws(p, e);
    if (p < e && *p == ',') {
      ++p;
      continue;
    }
    if (p < e && *p == '}') break;
    return false;
  }
  return have_img && have_shape;
}

// .npy (v1/v2/v3) uint8 C-order array -> shape + data pointer
bool parse_npy_u8(const char* b, size_t n, std::vector<long>& shape, const uint8_t** data, size_t* dn) {
  if (n < 12 || memcmp(b, "\x93NUMPY", 6) != 0) return false;
  const int major = (unsigned char)b[6];
  size_t hl, off;
  if (major == 1) {
    hl = (unsigned char)b[8] | (unsigned)(unsigned char)b[9] << 8;
    off = 10;
  } else {
    hl = (unsigned char)b[8] | (unsigned)(unsigned char)b[9] << 8 | (unsigned)(unsigned char)b[10] << 16 |
         (unsigned)(unsigned char)b[11] << 24;
    off = 12;
  }
  if (off + hl > n) return false;
  const std::string h(b + off, hl);
  if (h.find("'descr': '|u1'") == std::string::npos && h.find("'descr': '<u1'") == std::string::npos) return false;
  if (h.find("'fortran_order': False") == std::string::npos) return false;
  const size_t s0 = h.find("'shape': (");
  if (s0 == std::string::npos) return false;
  const char* p = h.c_str() + s0 + 10;
  for (;;) {
    while (*p == ' ') ++p;
    if (*p == ')') break;
    char* q;
    const long x = strtol(p, &q, 10);
    if (q == p) return false;
    shape.push_back(x);
    p = q;
    while (*p == ' ') ++p;
    if (*p == ',') ++p;
  }
  *data = reinterpret_cast<const uint8_t*>(b + off + hl);
  *dn = n - off - hl;
  return true;
}

// ---------------------------------------------------------------- the fast route
bool try_fast(Server* S, const std::string& method, const std::string& target, const std::string& ctype,
              const char* body, size_t blen, bool keep, std::string& out) {
  if (!S->has_fast.load(std::memory_order_acquire) || method != "POST") return false;
  std::string path = target, query;
  const size_t qpos = target.find('?');
  if (qpos != std::string::npos) {
    path = target.substr(0, qpos);
    query = target.substr(qpos + 1);
  }
  if (path != "/predict") return false;
  Fast f;
  {
    std::lock_guard<std::mutex> g(S->fast_mu);
    f = S->fast;
  }
  std::string qmodel;
  if (!query.empty()) {
    if (query.compare(0, 6, "model=") != 0 || query.find('&') != std::string::npos) return false;
    qmodel = query.substr(6);
  }
  const double t0 = now_ms();
  std::vector<long> shape;
  std::string model = qmodel;
  const size_t want = (size_t)f.H * f.W * f.C;
  thread_local std::vector<uint8_t> img;
  const uint8_t* src = nullptr;
  if (ctype.compare(0, 16, "application/json") == 0) {
    const char* b64;
    size_t b64n;
    std::string bm;
    if (!parse_json_image(body, blen, &b64, &b64n, shape, bm)) return false;
    if (!bm.empty()) model = bm;
    if (shape.size() == 4 && shape[0] == 1) shape.erase(shape.begin());
    if (shape.size() != 3 || shape[0] != f.H || shape[1] != f.W || shape[2] != f.C) return false;
    img.resize(want);
    if (!b64decode(b64, b64n, img.data(), want)) return false;
    src = img.data();
  } else if (ctype.compare(0, 24, "application/octet-stream") == 0) {
    const uint8_t* d;
    size_t dn;
    if (!parse_npy_u8(body, blen, shape, &d, &dn)) return false;
    if (shape.size() == 4 && shape[0] == 1) shape.erase(shape.begin());
    if (shape.size() != 3 || shape[0] != f.H || shape[1] != f.W || shape[2] != f.C || dn < want) return false;
    src = d;
  } else {
    return false;
  }
  if (!model.empty() && model != f.model) return false;
  const double t1 = now_ms();
  thread_local std::vector<float> y;
  y.resize(f.out_floats);
  double lat = 0;
  const void* ins[1] = {src};
  const int rc = hz_exec_submit(f.exec, ins, y.data(), &lat);
  const double t2 = now_ms();
  if (rc) {
    out = simple(503, "{\"error\": \"RuntimeError\", \"message\": \"executor request failed\"}", keep);
    return true;
  }
  // softmax (unless the plan emits probabilities) + top-5, as app.py does with numpy
  const int n = f.classes;
  thread_local std::vector<double> pr;
  pr.resize(n);
  if (f.probs) {
    for (int i = 0; i < n; ++i) pr[i] = y[i];
  } else {
    float m = -INFINITY;
    for (int i = 0; i < n; ++i) m = y[i] > m ? y[i] : m;
    double s = 0;
    for (int i = 0; i < n; ++i) s += (pr[i] = std::exp((double)y[i] - m));
    for (int i = 0; i < n; ++i) pr[i] /= s;
  }
  const int k = n < 5 ? n : 5;
  int top[5];
  for (int j = 0; j < k; ++j) {
    int best = -1;
    for (int i = 0; i < n; ++i) {
      bool used = false;
      for (int q = 0; q < j; ++q) used |= top[q] == i;
      if (!used && (best < 0 || pr[i] > pr[best])) best = i;
    }
    top[j] = best;
  }
  std::string js = "{\"model\": \"" + f.model + "\", \"backend\": \"gpu\", \"batch\": 1, \"top5\": [[";
  char tmp[64];
  for (int j = 0; j < k; ++j) {
    snprintf(tmp, sizeof(tmp), "%s[%d, %.6g]", j ? ", " : "", top[j], pr[top[j]]);
    js += tmp;
  }
  const double t3 = now_ms();
  snprintf(tmp, sizeof(tmp), "]], \"timing_ms\": %.3f}", t2 - t1);
  js += tmp;
  char h[400];
  snprintf(h, sizeof(h),
           "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n"
           "Access-Control-Allow-Origin: *\r\nAccess-Control-Expose-Headers: X-Timing\r\n"
           "X-Timing: decode=%.3f;infer=%.3f;total=%.3f\r\nX-Hipzap-Path: native\r\nConnection: %s\r\n\r\n",
           js.size(), t1 - t0, t2 - t1, t3 - t0, keep ? "keep-alive" : "close");
  out = std::string(h) + js;
  return true;
}

// ---------------------------------------------------------------- GET /inference
// an integer query value as Python's int() reads the plain forms ("[+-]digits"), at most 18
// digits (|x| < 2^63: the range the Flask route's engine call accepts; beyond it the Flask route
// answers, with its error), as two's complement mod 2^64 (the engine keeps seed & (2^62 - 1),
// which depends only on the value mod 2^62); false otherwise
bool parse_int(const std::string& v, unsigned long long* out, bool* neg) {
  size_t i = 0;
  *neg = false;
  if (i < v.size() && (v[i] == '+' || v[i] == '-')) *neg = v[i++] == '-';
  if (i == v.size() || v.size() - i > 18) return false;
  unsigned long long x = 0;
  for (; i < v.size(); ++i) {
    if (v[i] < '0' || v[i] > '9') return false;
    x = x * 10 + (unsigned long long)(v[i] - '0');
  }
  *out = *neg ? 0ull - x : x;
  return true;
}

bool try_lm(Server* S, const std::string& method, const std::string& target, bool keep, std::string& out) {
  if (method != "GET") return false;
  const size_t qpos = target.find('?');
  if (target.compare(0, qpos == std::string::npos ? target.size() : qpos, "/inference") != 0) return false;
  std::shared_ptr<const Lm> lm;
  {
    std::lock_guard<std::mutex> g(S->lm_mu);
    lm = S->lm;
  }
  if (!lm) return false;
  // only seed= / words= with plain integers; a prompt or anything else goes to the Flask route
  bool have_seed = false, have_words = false;
  unsigned long long seed = 0;
  int n = lm->dflt;
  if (qpos != std::string::npos) {
    const std::string q = target.substr(qpos + 1);
    size_t p = 0;
    while (p <= q.size()) {
      size_t e = q.find('&', p);
      if (e == std::string::npos) e = q.size();
      const std::string kv = q.substr(p, e - p);
      p = e + 1;
      if (kv.empty()) continue;
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) return false;
      const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
      unsigned long long x;
      bool neg;
      if (!parse_int(v, &x, &neg)) return false;
      if (k == "seed" && !have_seed) {
        have_seed = true;
        seed = x;
      } else if (k == "words" && !have_words && !neg && v.size() <= 9 && x >= 1 && x <= (unsigned long long)lm->maxn) {
        have_words = true;
        n = (int)x;
      } else {
        return false;  // (a repeated key, an out-of-range word count: the Flask route answers)
      }
    }
  }
  if (n < 1 || n > lm->maxn) return false;
  if (!have_seed) {
    thread_local std::mt19937_64 rng{std::random_device{}()};
    seed = rng();
  }
  seed &= (1ull << 62) - 1;
  const double t0 = now_ms();
  thread_local std::vector<int> ids;
  ids.resize(n);
  const int prompt = lm->empty_id;  // words = [""] (main.py:103)
  double lat = 0;
  const int rc = hz_lmb_submit(lm->sched, &prompt, 1, n, seed, ids.data(), nullptr, &lat);
  const double t1 = now_ms();
  if (rc) {
    out = simple(500, "{\"error\": \"RuntimeError\", \"message\": \"batched decode request failed\"}", keep);
    return true;
  }
  // the reference's detokenizer (serve/text.py Detokenizer, main.py:73-78): the prompt word "" adds
  // " "; a word after ".", "!" or a newline is capitalised; NO_SPACE words attach without a space
  std::string js = "{\"response\": {\"text\": \" ";
  js.reserve(16 + (size_t)n * 12);
  bool cap = false;
  for (int i = 0; i < n; ++i) {
    const int t = ids[i];
    if (t < 0 || t >= lm->V) {
      out = simple(500, "{\"error\": \"RuntimeError\", \"message\": \"token out of range\"}", keep);
      return true;
    }
    const uint8_t f = lm->fl[t];
    if (!(f & (cap ? 2 : 1))) js += ' ';
    js += cap ? lm->wc[t] : lm->w[t];
    cap = f & (cap ? 8 : 4);
  }
  js += "\"}}";
  const double t2 = now_ms();
  char h[400];
  snprintf(h, sizeof(h),
           "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n"
           "Access-Control-Allow-Origin: *\r\nAccess-Control-Expose-Headers: X-Timing\r\n"
           "X-Timing: generate=%.3f;detok=%.3f;total=%.3f\r\nX-Hipzap-Path: native\r\nConnection: %s\r\n\r\n",
           js.size(), t1 - t0, t2 - t1, t2 - t0, keep ? "keep-alive" : "close");
  out = std::string(h) + js;
  return true;
}

// ---------------------------------------------------------------- connections
// S->live was incremented by the spawner BEFORE this thread exists (hz_http_stop frees the server
// once it reads live == 0: a count taken here could come after that read)
void serve_conn(Server* S, int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  std::string buf;
  buf.reserve(1 << 18);
  char rd[65536];
  const size_t kMaxBody = size_t(64) << 20;
  bool open = true;
  while (open && !S->stop.load()) {
    // headers
    size_t hend;
    while ((hend = buf.find("\r\n\r\n")) == std::string::npos) {
      if (buf.size() > (1 << 16)) {
        open = false;
        break;
      }
      pollfd pf{fd, POLLIN, 0};
      const int pr = poll(&pf, 1, 250);
      if (S->stop.load()) {
        open = false;
        break;
      }
      if (pr == 0) continue;
      const ssize_t k = recv(fd, rd, sizeof(rd), 0);
      if (k <= 0) {
        open = false;
        break;
      }
      buf.append(rd, (size_t)k);
    }
    if (!open) break;
    const std::string head = buf.substr(0, hend);
    size_t le = head.find("\r\n");
    const std::string line = head.substr(0, le);
    const size_t sp1 = line.find(' '), sp2 = line.rfind(' ');
    if (sp1 == std::string::npos || sp2 == sp1) {
      send_str(fd, simple(400, "{\"error\": \"bad request line\"}", false));
      break;
    }
    const std::string method = line.substr(0, sp1), target = line.substr(sp1 + 1, sp2 - sp1 - 1),
                      version = line.substr(sp2 + 1);
    std::string headers = le == std::string::npos ? "" : head.substr(le + 2), ctype;
    long clen = 0;
    bool keep = version == "HTTP/1.1", chunked = false;
    {
      size_t p = 0;
      while (p < headers.size()) {
        size_t e = headers.find("\r\n", p);
        if (e == std::string::npos) e = headers.size();
        const std::string h = headers.substr(p, e - p);
        const size_t c = h.find(':');
        if (c != std::string::npos) {
          std::string k = h.substr(0, c), v = h.substr(c + 1);
          for (auto& ch : k) ch = (char)tolower(ch);
          while (!v.empty() && v[0] == ' ') v.erase(0, 1);
          if (k == "content-length") clen = atol(v.c_str());
          else if (k == "content-type") ctype = v;
          else if (k == "transfer-encoding") chunked = true;
          else if (k == "connection") {
            for (auto& ch : v) ch = (char)tolower(ch);
            if (v.find("close") != std::string::npos) keep = false;
            if (v.find("keep-alive") != std::string::npos) keep = true;
          }
        }
        p = e + 2;
      }
    }
    std::string resp;
    if (chunked || clen < 0 || (size_t)clen > kMaxBody) {
      S->n_bad++;
      send_str(fd, simple(chunked ? 411 : 413, "{\"error\": \"unsupported body framing\"}", false));
      break;
    }
    // body
    const size_t need = hend + 4 + (size_t)clen;
    while (buf.size() < need) {
      pollfd pf{fd, POLLIN, 0};
      const int pr = poll(&pf, 1, 250);
      if (S->stop.load()) {
        open = false;
        break;
      }
      if (pr == 0) continue;
      const ssize_t k = recv(fd, rd, sizeof(rd), 0);
      if (k <= 0) {
        open = false;
        break;
      }
      buf.append(rd, (size_t)k);
    }
    if (!open) break;
    const char* body = buf.data() + hend + 4;
    if (try_fast(S, method, target, ctype, body, (size_t)clen, keep, resp) || try_lm(S, method, target, keep, resp)) {
      S->n_fast++;
    } else if (S->py) {
      S->n_py++;
      PyReq r;
      r.keep = keep;
      S->py(&r, method.c_str(), target.c_str(), headers.c_str(), headers.size(), body, (uint64_t)clen);
      if (r.out.empty()) r.out = simple(500, "{\"error\": \"no response from the application\"}", keep);
      resp.swap(r.out);
    } else {
      resp = simple(404, "{\"error\": \"not found\"}", keep);
    }
    if (!send_all(fd, resp.data(), resp.size())) break;
    buf.erase(0, need);
    if (!keep) break;
  }
  close(fd);
  S->live--;
}

void accept_loop(Server* S) {
  while (!S->stop.load()) {
    pollfd pf{S->lfd, POLLIN, 0};
    const int pr = poll(&pf, 1, 250);
    if (pr <= 0) continue;
    const int fd = accept(S->lfd, nullptr, nullptr);
    if (fd < 0) continue;  // another process sharing the socket took it, or EINTR
    S->live++;
    std::thread(serve_conn, S, fd).detach();
  }
}

}  // namespace

extern "C" {

// listen_fd: a bound, listening TCP socket (the caller owns it; shared across worker processes)
void* hz_http_start(int listen_fd, PyHandler py) {
  auto* S = new Server();
  S->lfd = listen_fd;
  S->py = py;
  S->acceptor = std::thread(accept_loop, S);
  return S;
}

// the native POST /predict route over an executor (see hipzap/serve/native_http.py)
int hz_http_set_fast(void* h, void* exec, int H, int W, int C, int out_floats, int classes, int probs,
                     const char* model) {
  Server* S = static_cast<Server*>(h);
  if (!exec || H <= 0 || W <= 0 || C <= 0 || classes <= 0 || classes > out_floats) return -1;
  std::lock_guard<std::mutex> g(S->fast_mu);
  S->fast = Fast{exec, H, W, C, out_floats, classes, probs, model ? model : ""};
  S->has_fast.store(true, std::memory_order_release);
  return 0;
}

// the native GET /inference route over a decode scheduler (see hipzap/serve/native_http.py set_lm):
// blob = V entries of <JSON-escaped word>\0<JSON-escaped capitalised word>\0, flags[V] as struct Lm;
// sched = NULL removes the route
int hz_http_set_lm(void* h, void* sched, int V, int maxn, int dflt, int empty_id, const char* blob, uint64_t blen,
                   const uint8_t* flags) {
  Server* S = static_cast<Server*>(h);
  if (!sched) {
    std::lock_guard<std::mutex> g(S->lm_mu);
    S->lm.reset();
    return 0;
  }
  if (V < 1 || maxn < 1 || dflt < 1 || empty_id < 0 || empty_id >= V || !blob || !flags) return -1;
  auto lm = std::make_shared<Lm>();
  lm->sched = sched;
  lm->V = V;
  lm->maxn = maxn;
  lm->dflt = dflt;
  lm->empty_id = empty_id;
  lm->w.reserve(V);
  lm->wc.reserve(V);
  uint64_t p = 0;
  for (int i = 0; i < V; ++i) {
    for (int k = 0; k < 2; ++k) {
      const void* z = memchr(blob + p, 0, blen - p);
      if (p >= blen || !z) return -2;
      const uint64_t e = (uint64_t)(static_cast<const char*>(z) - blob);
      (k ? lm->wc : lm->w).emplace_back(blob + p, e - p);
      p = e + 1;
    }
  }
  if (p != blen) return -2;
  lm->fl.assign(flags, flags + V);
  std::lock_guard<std::mutex> g(S->lm_mu);
  S->lm = std::move(lm);
  return 0;
}

void hz_http_respond(void* req, int status, const char* headers, uint64_t hlen, const char* body, uint64_t blen) {
  PyReq* r = static_cast<PyReq*>(req);
  char line[64];
  snprintf(line, sizeof(line), "HTTP/1.1 %d %s\r\n", status, reason(status));
  r->out.assign(line);
  r->out.append(headers, hlen);  // "Name: value\r\n" lines incl. Content-Length
  r->out.append(r->keep ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
  r->out.append(body, blen);
}

void hz_http_stats(void* h, uint64_t* out4) {
  Server* S = static_cast<Server*>(h);
  out4[0] = S->n_fast.load();
  out4[1] = S->n_py.load();
  out4[2] = S->n_bad.load();
  out4[3] = (uint64_t)S->live.load();
}

// stop accepting, let open connections notice within one poll period, then free. Returns 1 when
// every connection thread has ended (the caller may then destroy the executor the fast route
// submits to), 0 when some are still live after 1 s: the server state is leaked and the caller
// must leak the executor too rather than free it under a connection inside hz_exec_submit.
int hz_http_stop(void* h) {
  Server* S = static_cast<Server*>(h);
  S->stop.store(true);
  if (S->acceptor.joinable()) S->acceptor.join();
  for (int i = 0; i < 100 && S->live.load() > 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  if (S->live.load() != 0) return 0;
  delete S;
  return 1;
}

}  // extern "C"
