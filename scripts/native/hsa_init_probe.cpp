// Cold-start decomposition probe (VERDICT r5 next #2b): in a fresh process, time the ROCr (HSA)
// layer's phases separately, then HIP's increment on top of an already initialised ROCr:
//   hsa_init                      -- KFD open, topology read, every visible agent's setup
//   agents + memory pools         -- hsa_iterate_agents + hsa_amd_agent_iterate_memory_pools
//   first hsa_queue_create        -- one AQL queue on the GPU agent (doorbell, ring buffer, CP map)
//   hipSetDevice + hipFree(0)     -- HIP's own runtime init over the live ROCr (its device objects,
//                                    code-object loader, its own queues are created lazily)
//   first hipStream + first op    -- HIP's first stream and a 4-KiB memset through it
// With ``--hip-only`` the HSA phases are skipped (HIP does all of it itself: the plain floor).
// Prints one JSON line; run it in >= 10 fresh processes per environment (scripts/cold_decompose.py).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Census {
  int agents = 0, gpus = 0, pools = 0;
  hsa_agent_t gpu{};
};

static hsa_status_t pool_cb(hsa_amd_memory_pool_t, void* d) {
  ++static_cast<Census*>(d)->pools;
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t agent_cb(hsa_agent_t a, void* d) {
  Census* c = static_cast<Census*>(d);
  ++c->agents;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU) {
    if (c->gpus == 0) c->gpu = a;
    ++c->gpus;
  }
  hsa_amd_agent_iterate_memory_pools(a, pool_cb, d);
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  const bool hip_only = argc > 1 && std::strcmp(argv[1], "--hip-only") == 0;
  // --null-first: HIP alone, then the first operation on the NULL stream before any stream exists
  // (is the default stream's hardware queue made at init, or lazily like a created stream's?)
  const bool null_first = argc > 1 && std::strcmp(argv[1], "--null-first") == 0;
  const double t0 = now_ms();
  Census c;
  double t_init = t0, t_enum = t0, t_queue = t0;
  hsa_queue_t* q = nullptr;
  if (null_first) {
    hipError_t e = hipSetDevice(0);
    if (e == hipSuccess) e = hipFree(nullptr);
    const double t_init_ = now_ms();
    void* p = nullptr;
    if (e == hipSuccess) e = hipMalloc(&p, 4096);
    const double t_mal = now_ms();
    if (e == hipSuccess) e = hipMemsetAsync(p, 0, 4096, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    const double t_null = now_ms();
    hipStream_t st = nullptr;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const double t_stream = now_ms();
    std::printf("{\"null_first\": true, \"hip_init_ms\": %.2f, \"malloc_ms\": %.2f, \"null_first_op_ms\": %.2f, "
                "\"then_stream_ms\": %.2f, \"total_ms\": %.2f, \"rc\": %d}\n",
                t_init_ - t0, t_mal - t_init_, t_null - t_mal, t_stream - t_null, t_stream - t0, (int)e);
    if (st) (void)hipStreamDestroy(st);
    if (p) (void)hipFree(p);
    return e == hipSuccess ? 0 : 1;
  }
  if (!hip_only) {
    if (hsa_init() != HSA_STATUS_SUCCESS) {
      std::printf("{\"error\": \"hsa_init failed\"}\n");
      return 1;
    }
    t_init = now_ms();
    hsa_iterate_agents(agent_cb, &c);
    t_enum = now_ms();
    if (c.gpus > 0 &&
        hsa_queue_create(c.gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q) !=
            HSA_STATUS_SUCCESS)
      q = nullptr;
    t_queue = now_ms();
  }
  hipError_t e = hipSetDevice(0);
  if (e == hipSuccess) e = hipFree(nullptr);
  const double t_hip = now_ms();
  hipStream_t st = nullptr;
  void* p = nullptr;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  const double t_stream = now_ms();
  if (e == hipSuccess) e = hipMalloc(&p, 4096);
  if (e == hipSuccess) e = hipMemsetAsync(p, 0, 4096, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  const double t_op = now_ms();
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  std::printf("{\"hip_only\": %s, \"hsa_init_ms\": %.2f, \"agents_pools_ms\": %.2f, \"queue_create_ms\": %.2f, "
              "\"hip_init_ms\": %.2f, \"first_stream_ms\": %.2f, \"first_op_ms\": %.2f, \"total_ms\": %.2f, "
              "\"agents\": %d, \"gpu_agents\": %d, \"pools\": %d, \"hip_devices\": %d, \"rc\": %d}\n",
              hip_only ? "true" : "false", t_init - t0, t_enum - t_init, t_queue - t_enum, t_hip - t_queue,
              t_stream - t_hip, t_op - t_stream, t_op - t0, c.agents, c.gpus, c.pools, ndev, (int)e);
  if (p) (void)hipFree(p);
  if (st) (void)hipStreamDestroy(st);
  if (q) hsa_queue_destroy(q);
  if (!hip_only) hsa_shut_down();
  return e == hipSuccess ? 0 : 1;
}
