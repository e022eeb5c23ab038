// Probe: how a tick reaches the GPU on MI355X — the dispatch mechanisms a per-tick kernel
// chain could use, each timed from the host's post to the host seeing the tick's completion
// flag (a system-scope store into pinned host memory, polled by the host: how the io loops
// take tick results), over N ticks:
//
//   launch1      hipLaunchKernelGGL of one fused kernel per tick
//   launch3      three dependent launches per tick (the K1 -> K2 -> K5 chain unfused)
//   graph1       hipGraphLaunch of a captured one-kernel graph (arguments fixed at capture:
//                the kernel reads the tick's descriptor from pinned memory, so nothing is
//                re-instantiated or updated per tick)
//   graph3       hipGraphLaunch of the captured three-kernel chain
//   graph1_upd   graph1 plus hipGraphExecKernelNodeSetParams per tick (new kernel arguments
//                every tick, as a one-shot launch passes them)
//   doorbell     a persistent one-wave kernel polling a host-mapped doorbell (the production
//                HipGrid path: no launch per tick at all)
//
// Each variant reports p10 / p50 / p90 of post -> completion seen, and the host CPU time of the
// post call itself (what the io loop pays).  Grids are 1 workgroup or 256 (one per CU) of 256
// threads.  Every kernel exits on a time limit (s_memrealtime) as well as on its stop word,
// and the persistent kernel's stream is synchronised before the process ends.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

struct Desc {
  uint32_t seq;   // the tick being posted
  uint32_t stop;  // doorbell kernel: exit
};

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// a stage of the chain: reads the tick's descriptor (host memory, system scope) and, last
// stage only, publishes completion to the host.  Block 0 / thread 0 does the work — the
// other workgroups only make the dispatch as wide as a production tick's.
__global__ void stage_k(const Desc* d, uint32_t* done, uint32_t* scratch, int last) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const uint32_t s = __hip_atomic_load(&d->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (last) {
    __hip_atomic_store(done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    scratch[0] = s;  // a dependent stage's output (device memory)
  }
}

// one-shot with the tick number as a kernel argument (graph1_upd / launch with arguments)
__global__ void stage_arg(uint32_t s, uint32_t* done) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  __hip_atomic_store(done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// persistent: one wave polls the doorbell until stop or the time limit
__global__ void doorbell_k(const Desc* d, uint32_t* done, uint64_t limit_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t last = 0;
  for (;;) {
    const uint32_t stop = __hip_atomic_load(&d->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (stop) return;
    const uint32_t s = __hip_atomic_load(&d->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s != last) {
      last = s;
      __hip_atomic_store(done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) return;
    __builtin_amdgcn_s_sleep(8);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Stat {
  std::vector<double> rtt, call;
};

static void report(const char* name, int grid, Stat& s) {
  if (s.rtt.size() < 10) {
    printf("{\"variant\": \"%s\", \"grid\": %d, \"error\": \"only %zu ticks completed\"}\n", name, grid, s.rtt.size());
    return;
  }
  std::sort(s.rtt.begin(), s.rtt.end());
  std::sort(s.call.begin(), s.call.end());
  const size_t n = s.rtt.size();
  printf("{\"variant\": \"%s\", \"grid\": %d, \"n\": %zu, \"post_to_done_p10_us\": %.2f, \"post_to_done_p50_us\": %.2f, "
         "\"post_to_done_p90_us\": %.2f, \"post_call_p50_us\": %.2f}\n",
         name, grid, n, s.rtt[n / 10], s.rtt[n / 2], s.rtt[n * 9 / 10], s.call[s.call.size() / 2]);
  fflush(stdout);
}

// post tick i with `post`, then spin on the completion flag (100 ms limit per tick)
template <class Post>
static bool run(Stat& st, Desc* h_desc, volatile uint32_t* h_done, int N, Post&& post) {
  for (int i = 1; i <= N + 20; ++i) {
    const double t0 = now_us();
    __atomic_store_n(&h_desc->seq, (uint32_t)i, __ATOMIC_RELEASE);
    if (!post(i)) return false;
    const double t1 = now_us();
    while (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != (uint32_t)i)
      if (now_us() - t0 > 100000) return false;
    const double t2 = now_us();
    if (i > 20) {  // warm-up excluded
      st.rtt.push_back(t2 - t0);
      st.call.push_back(t1 - t0);
    }
  }
  return true;
}

int main() {
  const int N = 2000;
  Desc* h_desc;
  uint32_t* h_done;
  uint32_t* d_scratch;
  CHECK(hipHostMalloc((void**)&h_desc, 4096, hipHostMallocMapped));
  CHECK(hipHostMalloc((void**)&h_done, 4096, hipHostMallocMapped));
  CHECK(hipMalloc((void**)&d_scratch, 4096));
  memset(h_desc, 0, 4096);
  memset(h_done, 0, 4096);
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  volatile uint32_t* done = h_done;

  for (int grid : {1, 256}) {
    const dim3 g(grid), b(256);
    {  // launch1
      Stat s;
      __atomic_store_n(h_done, 0u, __ATOMIC_RELEASE);
      bool ok = run(s, h_desc, done, N, [&](int) {
        hipLaunchKernelGGL(stage_k, g, b, 0, st, h_desc, h_done, d_scratch, 1);
        return true;
      });
      CHECK(hipStreamSynchronize(st));
      if (ok) report("launch1", grid, s);
    }
    {  // launch3
      Stat s;
      __atomic_store_n(h_done, 0u, __ATOMIC_RELEASE);
      bool ok = run(s, h_desc, done, N, [&](int) {
        hipLaunchKernelGGL(stage_k, g, b, 0, st, h_desc, h_done, d_scratch, 0);
        hipLaunchKernelGGL(stage_k, g, b, 0, st, h_desc, h_done, d_scratch, 0);
        hipLaunchKernelGGL(stage_k, g, b, 0, st, h_desc, h_done, d_scratch, 1);
        return true;
      });
      CHECK(hipStreamSynchronize(st));
      if (ok) report("launch3", grid, s);
    }
    for (int nk : {1, 3}) {  // graph1 / graph3: captured once, launched per tick
      hipGraph_t gr;
      hipGraphExec_t ex;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < nk; ++k)
        hipLaunchKernelGGL(stage_k, g, b, 0, st, h_desc, h_done, d_scratch, k == nk - 1 ? 1 : 0);
      CHECK(hipStreamEndCapture(st, &gr));
      CHECK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
      Stat s;
      __atomic_store_n(h_done, 0u, __ATOMIC_RELEASE);
      bool ok = run(s, h_desc, done, N, [&](int) { return hipGraphLaunch(ex, st) == hipSuccess; });
      CHECK(hipStreamSynchronize(st));
      if (ok) report(nk == 1 ? "graph1" : "graph3", grid, s);
      hipGraphExecDestroy(ex);
      hipGraphDestroy(gr);
    }
    {  // graph1_upd: new kernel arguments every tick
      hipGraph_t gr;
      hipGraphExec_t ex;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      hipLaunchKernelGGL(stage_arg, g, b, 0, st, 0u, h_done);
      CHECK(hipStreamEndCapture(st, &gr));
      CHECK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
      size_t nn = 0;
      CHECK(hipGraphGetNodes(gr, nullptr, &nn));
      std::vector<hipGraphNode_t> nodes(nn);
      CHECK(hipGraphGetNodes(gr, nodes.data(), &nn));
      Stat s;
      __atomic_store_n(h_done, 0u, __ATOMIC_RELEASE);
      uint32_t arg_s = 0;
      uint32_t* arg_done = h_done;
      void* args[] = {&arg_s, &arg_done};
      bool ok = nn == 1 && run(s, h_desc, done, N, [&](int i) {
        arg_s = (uint32_t)i;
        hipKernelNodeParams p{};
        p.func = (void*)stage_arg;
        p.gridDim = g;
        p.blockDim = b;
        p.sharedMemBytes = 0;
        p.kernelParams = args;
        p.extra = nullptr;
        if (hipGraphExecKernelNodeSetParams(ex, nodes[0], &p) != hipSuccess) return false;
        return hipGraphLaunch(ex, st) == hipSuccess;
      });
      CHECK(hipStreamSynchronize(st));
      if (ok) report("graph1_upd", grid, s);
      else printf("{\"variant\": \"graph1_upd\", \"grid\": %d, \"error\": \"update or launch failed\"}\n", grid);
      hipGraphExecDestroy(ex);
      hipGraphDestroy(gr);
    }
  }
  {  // doorbell: a persistent wave, on a stream of its own (highest priority: its own queue)
    int lo = 0, hi = 0;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t ps;
    CHECK(hipStreamCreateWithPriority(&ps, hipStreamNonBlocking, hi));
    __atomic_store_n(&h_desc->seq, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&h_desc->stop, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(h_done, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(doorbell_k, dim3(1), dim3(64), 0, ps, h_desc, h_done, (uint64_t)500000000ull /* 5 s */);
    Stat s;
    bool ok = run(s, h_desc, done, N, [&](int) { return true; });
    __atomic_store_n(&h_desc->stop, 1u, __ATOMIC_RELEASE);
    CHECK(hipStreamSynchronize(ps));
    if (ok) report("doorbell", 1, s);
    else printf("{\"variant\": \"doorbell\", \"error\": \"a tick was not answered\"}\n");
    hipStreamDestroy(ps);
  }
  hipStreamDestroy(st);
  return 0;
}
