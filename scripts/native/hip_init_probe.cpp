// Cold-start floor probe: time of the first HIP call (runtime + device init) in a fresh process,
// with and without libhipzap.so (7 MB of gfx950 code objects) loaded first.
//   hip_init_probe [path/to/libhipzap.so]
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const double t0 = now_ms();
  if (argc > 1 && !dlopen(argv[1], RTLD_NOW | RTLD_GLOBAL)) {
    std::printf("{\"error\": \"dlopen failed: %s\"}\n", dlerror());
    return 1;
  }
  const double t1 = now_ms();
  hipError_t e = hipSetDevice(0);
  if (e == hipSuccess) e = hipFree(nullptr);
  const double t2 = now_ms();
  void* p = nullptr;
  if (e == hipSuccess) e = hipMalloc(&p, 64 << 20);
  const double t3 = now_ms();
  hipStream_t st = nullptr;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  const double t4 = now_ms();
  if (e == hipSuccess) e = hipMemsetAsync(p, 0, 4096, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  const double t5 = now_ms();
  std::printf("{\"lib\": %s, \"dlopen_ms\": %.2f, \"hip_init_ms\": %.2f, \"malloc64MB_ms\": %.2f, "
              "\"first_stream_ms\": %.2f, \"first_op_ms\": %.2f, \"rc\": %d}\n",
              argc > 1 ? "true" : "false", t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, (int)e);
  if (st) (void)hipStreamDestroy(st);
  if (p) (void)hipFree(p);
  return e == hipSuccess ? 0 : 1;
}
