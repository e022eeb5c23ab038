// Probe: which HIP streams share a hardware queue with a persistent grid (MI355X).
//
// A persistent kernel holds its hardware queue: every packet queued behind it on the same
// queue waits until it exits.  HIP maps streams onto GPU_MAX_HW_QUEUES queues per priority
// and reuses the least-used queue once the pool is full, so which streams block behind the
// production grid (HipGrid) depends on how many streams the process created and with what
// priority.  This probe measures it:
//   * a "grid" kernel (one wave, spins on a host-mapped flag, exits on its own after 2 s of
//     device clock) runs on a stream created in MODE (normal / high / low priority / CU mask);
//   * NBEFORE normal streams are created before it and NAFTER after it (the production
//     worker creates engines' and the exchange's streams around the grid's);
//   * every stream — and the null stream (hipMemcpyAsync with stream 0) — gets a trivial
//     kernel; after 100 ms the probe records which completed while the grid still spins;
//   * then the flag releases the grid, and everything is synchronised.
// Output: one JSON line per mode.  A stream that did not complete shares the grid's queue.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void grid_spin(volatile uint32_t* flag, uint32_t* started, uint64_t limit_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(started, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (__hip_atomic_load((uint32_t*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ void touch(uint32_t* out, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(out, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void run(const std::string& mode, int nbefore, int nafter) {
  uint32_t *flag = nullptr, *started = nullptr, *marks = nullptr;
  const int n = nbefore + nafter;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocMapped));
  CK(hipHostMalloc((void**)&started, 64, hipHostMallocMapped));
  CK(hipHostMalloc((void**)&marks, 4 * (n + 2), hipHostMallocMapped));
  *flag = 0;
  *started = 0;
  std::memset(marks, 0, 4 * (n + 2));
  uint32_t* d_buf = nullptr;
  CK(hipMalloc((void**)&d_buf, 4096));
  std::vector<uint32_t> hbuf(1024);

  std::vector<hipStream_t> st(n);
  for (int i = 0; i < nbefore; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  hipStream_t g = nullptr;
  if (mode == "normal") {
    CK(hipStreamCreateWithFlags(&g, hipStreamNonBlocking));
  } else if (mode == "high" || mode == "low") {
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&g, hipStreamNonBlocking, mode == "high" ? greatest : least));
  } else if (mode == "cumask") {
    hipDeviceProp_t pr{};
    CK(hipGetDeviceProperties(&pr, 0));
    std::vector<uint32_t> m((pr.multiProcessorCount + 31) / 32, 0xffffffffu);
    CK(hipExtStreamCreateWithCUMask(&g, (uint32_t)m.size(), m.data()));
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    exit(2);
  }
  for (int i = nbefore; i < n; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));

  hipLaunchKernelGGL(grid_spin, dim3(1), dim3(64), 0, g, flag, started, (uint64_t)200000000ull /* 2 s */);
  CK(hipGetLastError());
  const double t0 = now_ms();
  while (!__atomic_load_n(started, __ATOMIC_ACQUIRE))
    if (now_ms() - t0 > 1000) break;
  const bool grid_started = __atomic_load_n(started, __ATOMIC_ACQUIRE) != 0;

  for (int i = 0; i < n; ++i) {
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st[i], marks + i, 1u);
    CK(hipGetLastError());
  }
  // the null stream: an asynchronous copy (what a synchronous hipMemcpy would wait behind)
  hipEvent_t ev_null;
  CK(hipEventCreateWithFlags(&ev_null, hipEventDisableTiming));
  CK(hipMemcpyAsync(hbuf.data(), d_buf, 4096, hipMemcpyDeviceToHost, 0));
  CK(hipEventRecord(ev_null, 0));
  // a copy on a stream of its own (the exchange's copy-after-round path)
  hipStream_t cs;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipEvent_t ev_copy;
  CK(hipEventCreateWithFlags(&ev_copy, hipEventDisableTiming));
  CK(hipMemcpyAsync(hbuf.data(), d_buf, 4096, hipMemcpyDeviceToHost, cs));
  CK(hipEventRecord(ev_copy, cs));

  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  std::string blocked;
  int nblocked = 0;
  for (int i = 0; i < n; ++i)
    if (!__atomic_load_n(marks + i, __ATOMIC_ACQUIRE)) {
      blocked += (blocked.empty() ? "" : ",") + std::to_string(i);
      ++nblocked;
    }
  const bool null_done = hipEventQuery(ev_null) == hipSuccess;
  const bool copy_done = hipEventQuery(ev_copy) == hipSuccess;
  const bool grid_still = hipStreamQuery(g) == hipErrorNotReady;

  __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);
  CK(hipDeviceSynchronize());
  const char* hq = getenv("GPU_MAX_HW_QUEUES");
  printf("{\"mode\": \"%s\", \"gpu_max_hw_queues\": \"%s\", \"streams_before\": %d, \"streams_after\": %d, "
         "\"grid_started\": %s, \"grid_still_running_at_check\": %s, \"blocked_streams\": [%s], \"n_blocked\": %d, "
         "\"null_stream_copy_done\": %s, \"own_stream_copy_done\": %s}\n",
         mode.c_str(), hq ? hq : "(unset)", nbefore, nafter, grid_started ? "true" : "false",
         grid_still ? "true" : "false", blocked.c_str(), nblocked, null_done ? "true" : "false",
         copy_done ? "true" : "false");
  fflush(stdout);
  for (auto s : st) CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(g));
  CK(hipStreamDestroy(cs));
  CK(hipEventDestroy(ev_null));
  CK(hipEventDestroy(ev_copy));
  CK(hipFree(d_buf));
  CK(hipHostFree(flag));
  CK(hipHostFree(started));
  CK(hipHostFree(marks));
}

int main(int argc, char** argv) {
  // queue_probe MODE NBEFORE NAFTER  (one mode per process: HIP's queue pool is per process)
  const std::string mode = argc > 1 ? argv[1] : "normal";
  const int nb = argc > 2 ? atoi(argv[2]) : 6, na = argc > 3 ? atoi(argv[3]) : 6;
  CK(hipSetDevice(0));
  run(mode, nb, na);
  return 0;
}
