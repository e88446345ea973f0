// hipzap-serve-plan: a Python-free serving process for a vision plan image (.hzplan).
//
//   hipzap-serve-plan PLAN [--port 8080] [--host 127.0.0.1] [--contexts 24] [--device 0] [--max-wait-us 200]
//   (a plan exported with --batch B > 1 is served with dynamic batching: each POST is one image)
//   hipzap-serve-plan PLAN --once IMAGE.raw      (cold-start probe: one request, JSON to stdout)
//
// The same native pieces the Python server composes (csrc/plan.cpp loader, csrc/executor.cpp
// request executor, csrc/http.cpp HTTP/1.1 front end with the POST /predict fast route), in
// one executable: no interpreter start, no imports, so the serverless cold path is exec -> HIP
// init -> plan upload -> first request. GET /health answers {"status": "ok", ...}; every other
// route that is not the fast POST /predict gets a JSON 404 (the full Flask app -- /inference,
// /metrics, CORS preflight -- stays in `python -m hipzap serve`).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../hipzap.h"

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop.store(true); }

// The plan's JSON metadata is written by engine/plan.py with json.dumps defaults, so the few
// fields needed here are found by key after the section they belong to.
bool num_after(const std::string& js, size_t from, const char* key, long long& out) {
  const size_t k = js.find(std::string("\"") + key + "\": ", from);
  if (k == std::string::npos) return false;
  out = std::atoll(js.c_str() + k + std::strlen(key) + 4);
  return true;
}

struct Spec {
  long long in_off = 0, in_bytes = 0, out_off = 0, out_bytes = 0, classes = 0, H = 0, W = 0, C = 0;
  long long rows = 1;  // plan batch: > 1 -> dynamic batching of one-image requests
  int probs = 0;
  std::string model;
  bool host_io = false;
};

bool read_spec(const char* path, Spec& s) {
  std::ifstream f(path, std::ios::binary);
  char hdr[128];
  if (!f.read(hdr, sizeof(hdr)) || std::memcmp(hdr, "HZPLAN01", 8) != 0) return false;
  uint64_t meta_off, meta_len;
  std::memcpy(&meta_off, hdr + 32, 8);
  std::memcpy(&meta_len, hdr + 40, 8);
  std::string js(meta_len, '\0');
  f.seekg((std::streamoff)meta_off);
  if (!f.read(&js[0], (std::streamsize)meta_len)) return false;
  const size_t mi = js.find("\"model\": \"");
  if (mi != std::string::npos) s.model = js.substr(mi + 10, js.find('"', mi + 10) - (mi + 10));
  s.probs = js.find("\"probs\": true") != std::string::npos;
  s.host_io = js.find("\"host_io\": true") != std::string::npos;
  const size_t ii = js.find("\"inputs\": [");
  const size_t oi = js.find("\"output\": {");
  if (ii == std::string::npos || oi == std::string::npos) return false;
  if (!num_after(js, ii, "off", s.in_off) || !num_after(js, ii, "bytes", s.in_bytes)) return false;
  const size_t sh = js.find("\"shape\": [", ii);
  if (sh == std::string::npos || sh > oi) return false;
  long long d[4] = {0, 0, 0, 0};
  if (std::sscanf(js.c_str() + sh + 10, "%lld, %lld, %lld, %lld", &d[0], &d[1], &d[2], &d[3]) != 4) return false;
  s.rows = d[0], s.H = d[1], s.W = d[2], s.C = d[3];  // uint8 input [B][H][W][C], one image per request
  if (!num_after(js, oi, "off", s.out_off) || !num_after(js, oi, "bytes", s.out_bytes)) return false;
  if (!num_after(js, oi, "num_labels", s.classes) || s.classes <= 0) s.classes = s.out_bytes / 4 / (d[0] > 0 ? d[0] : 1);
  return d[0] >= 1 && s.in_bytes == d[0] * d[1] * d[2] * d[3] && s.out_bytes % d[0] == 0;
}

void fallback(void* req, const char* method, const char* target, const char*, uint64_t, const char*, uint64_t);
std::string g_health;

void fallback(void* req, const char* method, const char* target, const char*, uint64_t, const char*, uint64_t) {
  std::string body, hdr;
  int status = 200;
  if (!std::strcmp(method, "GET") && (!std::strcmp(target, "/health") || !std::strncmp(target, "/health?", 8))) {
    body = g_health;
  } else {
    status = 404;
    body = "{\"error\": \"not found (hipzap-serve-plan serves POST /predict and GET /health)\"}";
  }
  hdr = "Content-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  hz_http_respond(req, status, hdr.data(), hdr.size(), body.data(), body.size());
}

int die(const char* what) {
  std::fprintf(stderr, "hipzap-serve-plan: %s: %s\n", what, hz_plan_last_error());
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  const double t0 = now_ms();
  // blit-kernel copies instead of SDMA unless the deployment chose (hipzap/lite.py no_sdma_default:
  // faster weight upload and first queue; the request path has no copies)
  const char* keep = std::getenv("HIPZAP_KEEP_SDMA");
  if (!keep || std::strcmp(keep, "1") != 0) setenv("HSA_ENABLE_SDMA", "0", 0);
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s PLAN [--port P] [--host H] [--contexts N] [--device D] [--max-wait-us U] [--once IMAGE]\n", argv[0]);
    return 2;
  }
  const char* plan_path = argv[1];
  int port = 8080, contexts = 24, device = 0;
  double max_wait_us = 200.0;
  std::string host = "127.0.0.1";
  const char* once = nullptr;
  for (int i = 2; i + 1 < argc; i += 2) {
    const std::string a = argv[i];
    if (a == "--port") port = std::atoi(argv[i + 1]);
    else if (a == "--host") host = argv[i + 1];
    else if (a == "--contexts") contexts = std::atoi(argv[i + 1]);
    else if (a == "--device") device = std::atoi(argv[i + 1]);
    else if (a == "--max-wait-us") max_wait_us = std::atof(argv[i + 1]);
    else if (a == "--once") once = argv[i + 1];
  }
  Spec sp;
  if (!read_spec(plan_path, sp) || !sp.host_io) {
    std::fprintf(stderr, "hipzap-serve-plan: %s is not a single-uint8-image host-I/O plan\n", plan_path);
    return 1;
  }
  double tm[HZ_PLAN_NT] = {0};
  void* plan = hz_plan_open(plan_path, device, 1, tm);
  if (!plan) return die("plan open");

  if (once) {  // cold-start probe: one request on one eagerly run (uncaptured) context
    std::ifstream f(once, std::ios::binary);
    std::vector<char> img((size_t)sp.in_bytes);
    if (!f.read(img.data(), (std::streamsize)img.size())) {
      std::fprintf(stderr, "hipzap-serve-plan: %s: need %lld bytes\n", once, sp.in_bytes);
      return 1;
    }
    const double t1 = now_ms();
    if (hz_plan_add_contexts(plan, 1, 0)) return die("context");
    std::vector<float> out((size_t)(sp.out_bytes / 4));
    if (hz_plan_infer(plan, 0, img.data(), (uint64_t)sp.in_off, (uint64_t)sp.in_bytes, out.data(),
                      (uint64_t)sp.out_off, (uint64_t)sp.out_bytes))
      return die("infer");
    const double t2 = now_ms();
    // wall clock of the first logits: the parent (hipzap/coldstart.py) subtracts its spawn time
    const double t_first = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    int best = 0;
    for (int i = 1; i < (int)sp.classes; ++i)
      if (out[i] > out[best]) best = i;
    std::printf("{\"mode\": \"native\", \"t_first\": %.6f, \"main_to_logits_ms\": %.2f, \"first_request_ms\": %.2f, \"argmax\": %d, "
                "\"logit0\": %.6g, \"phases_ms\": {\"parse\": %.2f, \"hip_init\": %.2f, \"upload\": %.2f, "
                "\"blob_alloc\": %.2f}}\n",
                t_first, t2 - t0, t2 - t1, best, out[0], tm[HZ_PLAN_T_PARSE], tm[HZ_PLAN_T_HIP_INIT], tm[HZ_PLAN_T_UPLOAD],
                tm[HZ_PLAN_T_BLOB_ALLOC]);
    std::fflush(stdout);
    hz_plan_close(plan);
    return 0;
  }

  {  // HIPZAP_STREAM_KIND=hiprio: contexts after the first on highest-priority streams (opt-in: a
     // mix of one normal- and several high-priority queues measured slower, profiles/r6_queues)
    const char* k = std::getenv("HIPZAP_STREAM_KIND");
    if (k && std::string(k) == "hiprio") hz_plan_set_stream_priority(plan, 1);
  }
  if (hz_plan_add_contexts(plan, contexts, 1)) return die("contexts");
  std::vector<HzProgram> progs(contexts);
  std::vector<hipStream_t> streams(contexts);
  std::vector<void*> ins(contexts), outs(contexts);
  for (int i = 0; i < contexts; ++i) {
    progs[i] = hz_plan_prog(plan, i);
    streams[i] = static_cast<hipStream_t>(hz_plan_stream(plan, i));
    ins[i] = static_cast<char*>(hz_plan_host(plan, i)) + sp.in_off;
    outs[i] = static_cast<char*>(hz_plan_host(plan, i)) + sp.out_off;
  }
  const uint64_t in_bytes = (uint64_t)sp.in_bytes;
  // a batch-B plan serves one-image requests with dynamic batching (csrc/executor.cpp)
  void* ex = sp.rows > 1 ? hz_exec_create_batched(progs.data(), streams.data(), ins.data(), &in_bytes, 1, outs.data(),
                                                  (uint64_t)sp.out_bytes, contexts, (int)sp.rows, max_wait_us, 1)
                         : hz_exec_create(progs.data(), streams.data(), ins.data(), &in_bytes, 1, outs.data(),
                                          (uint64_t)sp.out_bytes, contexts);
  if (!ex) return die("executor");

  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  const int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1 || bind(fd, (sockaddr*)&addr, sizeof(addr)) != 0 ||
      listen(fd, 1024) != 0) {
    std::perror("hipzap-serve-plan: bind/listen");
    return 1;
  }
  std::ostringstream hs;
  hs << "{\"status\": \"ok\", \"server\": \"hipzap-serve-plan\", \"model\": \"" << sp.model
     << "\", \"contexts\": " << contexts << ", \"device\": " << device << "}";
  g_health = hs.str();
  void* srv = hz_http_start(fd, fallback);
  if (!srv) {
    std::fprintf(stderr, "hipzap-serve-plan: HTTP server start failed\n");
    return 1;
  }
  if (hz_http_set_fast(srv, ex, (int)sp.H, (int)sp.W, (int)sp.C, (int)(sp.out_bytes / sp.rows / 4), (int)sp.classes, sp.probs,
                       sp.model.c_str())) {
    std::fprintf(stderr, "hipzap-serve-plan: fast route rejected (image %lldx%lldx%lld, %lld classes, %lld output bytes)\n",
                 sp.H, sp.W, sp.C, sp.classes, sp.out_bytes);
    hz_http_stop(srv);
    return 1;
  }
  std::fprintf(stderr, "hipzap-serve-plan: %s on http://%s:%d (%d contexts, ready in %.0f ms)\n", sp.model.c_str(),
               host.c_str(), port, contexts, now_ms() - t0);
  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  while (!g_stop.load()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  const int drained = hz_http_stop(srv);
  close(fd);
  if (drained) {  // else a connection may still be inside hz_exec_submit: the process exits instead
    hz_exec_destroy(ex);
    hz_plan_close(plan);
  }
  return 0;
}
