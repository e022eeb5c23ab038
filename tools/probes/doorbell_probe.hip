// Probe: host <-> GPU signalling round trip on MI355X, the loop-tick grid's doorbell path.
// One persistent wave ping-pongs with the host N times:
//   host: store in = i (release)          GPU: poll `in` until i, then store out = i (system)
//   host: spin until out == i -> RTT
// Doorbell placements for `in`:
//   host   pinned host memory, mapped (what HipGrid uses: every poll is a PCIe read)
//   dev    fine-grained device memory the CPU writes through the BAR (the GPU polls HBM)
// `out` is always pinned host memory (the host polls its own memory).  Each kernel has a
// time limit (s_memrealtime) so every wave exits even if the host stops answering.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void pingpong(volatile uint32_t* in, uint32_t* out, int n, uint64_t limit_ticks, int sleep) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 1; i <= n; ++i) {
    for (;;) {
      const uint32_t v = __hip_atomic_load((uint32_t*)in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == (uint32_t)i) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) return;
      if (sleep) __builtin_amdgcn_s_sleep(8);
    }
    __hip_atomic_store(out, (uint32_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void run(const char* name, uint32_t* in_host_ptr, uint32_t* in_dev_ptr, uint32_t* out, int sleep) {
  const int N = 2000;
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  __atomic_store_n(in_host_ptr, 0u, __ATOMIC_RELEASE);
  __atomic_store_n(out, 0u, __ATOMIC_RELEASE);
  hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, st, (volatile uint32_t*)in_dev_ptr, out, N,
                     (uint64_t)200000000ull /* 2 s */, sleep);
  std::vector<double> rtt;
  for (int i = 1; i <= N; ++i) {
    const double t0 = now_us();
    __atomic_store_n(in_host_ptr, (uint32_t)i, __ATOMIC_RELEASE);
    bool ok = true;
    while (__atomic_load_n(out, __ATOMIC_ACQUIRE) != (uint32_t)i)
      if (now_us() - t0 > 100000) {
        ok = false;
        break;
      }
    if (!ok) {
      printf("%s: no answer at %d\n", name, i);
      break;
    }
    rtt.push_back(now_us() - t0);
  }
  hipStreamSynchronize(st);
  hipStreamDestroy(st);
  if (rtt.size() < 100) return;
  std::sort(rtt.begin() + 0, rtt.end());
  printf("{\"doorbell\": \"%s\", \"sleep\": %d, \"n\": %zu, \"rtt_p50_us\": %.2f, \"rtt_p10_us\": %.2f, \"rtt_p90_us\": %.2f}\n",
         name, sleep, rtt.size(), rtt[rtt.size() / 2], rtt[rtt.size() / 10], rtt[rtt.size() * 9 / 10]);
}

int main() {
  uint32_t *h_in, *h_out;
  hipHostMalloc((void**)&h_in, 4096, hipHostMallocMapped);
  hipHostMalloc((void**)&h_out, 4096, hipHostMallocMapped);
  memset(h_in, 0, 4096);
  memset(h_out, 0, 4096);
  for (int sl : {1, 0}) run("host", h_in, h_in, h_out, sl);
  // fine-grained device memory: can the CPU write it (large BAR)?  hipPointerGetAttributes
  // says where it lives; a CPU store to an unmapped address would fault the probe (CPU-side)
  uint32_t* d_in = nullptr;
  if (hipExtMallocWithFlags((void**)&d_in, 4096, hipDeviceMallocFinegrained) == hipSuccess && d_in) {
    hipPointerAttribute_t a{};
    hipPointerGetAttributes(&a, d_in);
    printf("{\"finegrained_device\": true, \"type\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}\n",
           (int)a.type, a.hostPointer, a.devicePointer);
    fflush(stdout);
    if (a.hostPointer) {
      hipMemset(d_in, 0, 4096);
      hipDeviceSynchronize();
      for (int sl : {1, 0}) run("dev", (uint32_t*)a.hostPointer, d_in, h_out, sl);
    } else {
      printf("{\"note\": \"no host mapping for fine-grained device memory\"}\n");
    }
  }
  return 0;
}
