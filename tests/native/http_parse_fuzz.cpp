// Host ASan/UBSan fuzz of the native HTTP front end's parsers and request framing
// (hipzap/csrc/http.cpp, tests/test_native_asan_cpu.py). The translation unit is included so the
// anonymous-namespace parsers are reachable; every input lives in an exact-size heap buffer, so
// any read past the body is an ASan heap-buffer-overflow. serve_conn() is driven over a
// socketpair with random and mutated requests (no fast route, no Python handler: 404/400/413/411
// answers), including pipelined requests and truncated bodies.
#include "../../hipzap/csrc/http.cpp"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/time.h>

#include <atomic>
#include <vector>

#include <cstdlib>
#include <random>

extern "C" int hz_exec_submit(void*, const void* const*, void*, double*) { return 1; }
// the decode scheduler of the GET /inference route: deterministic token ids from the seed
extern "C" int hz_lmb_submit(void*, const int* prompt, int P, int n, unsigned long long seed, int* out, float*,
                             double* lat) {
  if (!prompt || P != 1 || n < 1 || !out) return -1;
  for (int i = 0; i < n; ++i) out[i] = (int)((seed * 2654435761ull + (unsigned long long)i * 7) % 6);
  if (lat) *lat = 1.0;
  return 0;
}

namespace {

std::mt19937_64 rng(12345);

std::string rnd_bytes(size_t n, const char* alphabet = nullptr) {
  std::string s(n, '\0');
  const size_t an = alphabet ? strlen(alphabet) : 0;
  for (auto& c : s) c = alphabet ? alphabet[rng() % an] : (char)(rng() & 0xff);
  return s;
}

std::string mutate(std::string s) {
  const int k = 1 + (int)(rng() % 4);
  for (int i = 0; i < k && !s.empty(); ++i) {
    const size_t at = rng() % s.size();
    switch (rng() % 4) {
      case 0: s[at] = (char)(rng() & 0xff); break;
      case 1: s.erase(at, 1 + rng() % 8); break;
      case 2: s.insert(at, rnd_bytes(1 + rng() % 8, "0123456789[]{},:\"' -+")); break;
      default: s.resize(at); break;
    }
  }
  return s;
}

template <class F>
void on_exact(const std::string& s, F f) {  // the input in a heap block of exactly its size
  char* b = static_cast<char*>(malloc(s.size() ? s.size() : 1));
  memcpy(b, s.data(), s.size());
  f(b, s.size());
  free(b);
}

void fuzz_parsers() {
  const std::string seeds[] = {
      "{\"image_b64\": \"AAECAwQF\", \"shape\": [1, 2, 3], \"model\": \"resnet50\"}",
      "{\"shape\": [224, 224, 3], \"image_b64\": \"////\"}",
      std::string("\x93NUMPY\x01\x00\x46\x00{'descr': '|u1', 'fortran_order': False, 'shape': (2, 3, 1), }      \n",
                  80) + "abcdef",
      std::string("\x93NUMPY\x02\x00\x10\x00\x00\x00{'shape': (5,", 26),
  };
  for (int it = 0; it < 200000; ++it) {
    std::string in = it % 5 == 4 ? rnd_bytes(rng() % 96, nullptr) : mutate(seeds[rng() % 4]);
    on_exact(in, [](const char* b, size_t n) {
      const char* img;
      size_t img_n;
      std::vector<long> shape;
      std::string model;
      if (parse_json_image(b, n, &img, &img_n, shape, model)) {
        if (img < b || img + img_n > b + n) abort();
        std::vector<uint8_t> out(img_n);
        b64decode(img, img_n, out.data(), (img_n * 3) / 4);
      }
      std::vector<long> s2;
      const uint8_t* d;
      size_t dn;
      if (parse_npy_u8(b, n, s2, &d, &dn) && (reinterpret_cast<const char*>(d) < b || reinterpret_cast<const char*>(d) + dn != b + n))
        abort();
      const char* p = b;
      std::vector<long> v;
      json_int_array(p, b + n, v);
      if (p < b || p > b + n) abort();
    });
  }
}

void fuzz_framing() {
  Server S;  // no fast route, no Python handler
  const std::string seeds[] = {
      "GET /health HTTP/1.1\r\nHost: x\r\n\r\n",
      "POST /predict HTTP/1.1\r\nContent-Type: application/json\r\nContent-Length: 13\r\n\r\n{\"a\": [1, 2]}",
      "POST /p HTTP/1.1\r\nContent-Length: 4\r\nConnection: keep-alive\r\n\r\nabcdGET / HTTP/1.1\r\n\r\n",
      "POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n",
      "POST / HTTP/1.0\r\nContent-Length: -7\r\n\r\n",
  };
  for (int it = 0; it < 4000; ++it) {
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) abort();
    std::string req = it % 7 == 6 ? rnd_bytes(rng() % 300, nullptr) : mutate(seeds[rng() % 5]);
    if (rng() % 3 == 0) req += seeds[rng() % 5];
    S.live++;  // the spawner's count (accept_loop)
    std::thread t(serve_conn, &S, sv[1]);  // closes sv[1] when it returns
    send_all(sv[0], req.data(), req.size());
    shutdown(sv[0], SHUT_WR);  // EOF: a truncated body ends the connection
    char sink[4096];
    while (recv(sv[0], sink, sizeof(sink), 0) > 0) {
    }
    t.join();
    close(sv[0]);
  }
}

// the GET /inference route: query strings fuzzed (seed / words / other keys, signs, overflow,
// repeats) through try_lm against a 6-word table; a request the route takes must produce a body
// of exactly n words from the table, and anything else must fall back (return false)
void fuzz_lm_route() {
  Server S;
  // words: "a", "B", ".", "n't", "q\"t", "\n" (JSON-escaped forms as Python writes them)
  const char* w[6] = {"a", "b", ".", "n't", "q\\\"t", "\\n"};
  const char* wc[6] = {"A", "B", ".", "N't", "Q\\\"t", "\\n"};
  std::string blob;
  for (int i = 0; i < 6; ++i) {
    blob += w[i];
    blob.push_back('\0');
    blob += wc[i];
    blob.push_back('\0');
  }
  const uint8_t fl[6] = {0, 0, 1 | 2 | 4 | 8, 1, 0, 4 | 8};
  int dummy = 0;
  if (hz_http_set_lm(&S, &dummy, 6, 50, 20, 0, blob.data(), blob.size(), fl) != 0) abort();
  if (hz_http_set_lm(&S, &dummy, 6, 50, 20, 7, blob.data(), blob.size(), fl) != -1) abort();  // empty id past V
  if (hz_http_set_lm(&S, &dummy, 7, 50, 20, 0, blob.data(), blob.size(), fl) != -2) abort();  // short blob
  const std::string seeds[] = {"/inference", "/inference?seed=5", "/inference?seed=-5&words=7",
                               "/inference?words=50&seed=999999999999999999", "/inference?words=0",
                               "/inference?prompt=a&seed=1", "/inference?seed=1&seed=2", "/inference?words=9999999999"};
  int native = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string t = it % 3 == 0 ? mutate(seeds[rng() % 8]) : seeds[rng() % 8];
    std::string out;
    if (try_lm(&S, "GET", t, true, out)) {
      ++native;
      const size_t b = out.find("\r\n\r\n");
      if (b == std::string::npos || out.compare(0, 15, "HTTP/1.1 200 OK") != 0) abort();
      const std::string body = out.substr(b + 4);
      if (body.compare(0, 23, "{\"response\": {\"text\": \"") != 0 || body.compare(body.size() - 3, 3, "\"}}") != 0)
        abort();
    }
  }
  std::string out;
  if (!try_lm(&S, "GET", "/inference?seed=3&words=4", true, out) || try_lm(&S, "POST", "/inference", true, out) ||
      try_lm(&S, "GET", "/inference?words=51", true, out) || try_lm(&S, "GET", "/inference?seed=1&x=2", true, out) ||
      try_lm(&S, "GET", "/inferencex", true, out))
    abort();
  if (hz_http_set_lm(&S, nullptr, 0, 0, 0, 0, nullptr, 0, nullptr) != 0 || try_lm(&S, "GET", "/inference", true, out))
    abort();  // route removed
  printf("lm route fuzz: %d native\n", native);
}

extern "C" void echo_handler(void* req, const char*, const char* target, const char*, uint64_t, const char*,
                             uint64_t blen) {
  const std::string body = std::string("{\"target\": \"") + target + "\", \"n\": " + std::to_string(blen) + "}";
  const std::string hdr = "Content-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  hz_http_respond(req, 200, hdr.data(), hdr.size(), body.data(), body.size());
}

// the whole server over loopback TCP: acceptor + one thread per connection + the handler
// callback, with hz_http_stop racing clients that are still connecting (5 start/stop rounds on
// one listening socket). Under ThreadSanitizer this is the race check of the connection
// accounting that lets hz_http_stop free the server.
void server_rounds() {
  const int lfd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  if (lfd < 0 || bind(lfd, (sockaddr*)&a, sizeof(a)) || listen(lfd, 256)) abort();
  socklen_t al = sizeof(a);
  getsockname(lfd, (sockaddr*)&a, &al);
  std::atomic<int> ok{0};
  for (int round = 0; round < 5; ++round) {
    void* srv = hz_http_start(lfd, echo_handler);
    std::atomic<bool> quit{false};
    std::vector<std::thread> cl;
    for (int c = 0; c < 6; ++c)
      cl.emplace_back([&, c] {
        while (!quit.load()) {
          const int fd = socket(AF_INET, SOCK_STREAM, 0);
          timeval tv{0, 200000};
          setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
          if (connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
            const std::string req = "POST /c" + std::to_string(c) +
                                    " HTTP/1.1\r\nContent-Length: 3\r\nConnection: close\r\n\r\nabc";
            send_all(fd, req.data(), req.size());
            char buf[512];
            const ssize_t k = recv(fd, buf, sizeof(buf) - 1, 0);
            if (k > 0) {
              buf[k] = 0;
              if (strstr(buf, "200 OK") && strstr(buf, "\"n\": 3")) ok++;
            }
          }
          close(fd);
        }
      });
    std::this_thread::sleep_for(std::chrono::milliseconds(60));
    const int freed = hz_http_stop(srv);  // clients are still connecting
    quit.store(true);
    for (auto& t : cl) t.join();
    if (!freed) abort();  // every connection here is short: the server must have been freed
  }
  close(lfd);
  if (ok.load() < 10) abort();
  printf("server rounds: %d answered\n", ok.load());
}

}  // namespace

int main() {
  fuzz_parsers();
  fuzz_framing();
  fuzz_lm_route();
  server_rounds();
  printf("http parse fuzz: ok\n");
  return 0;
}
