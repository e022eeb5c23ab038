// Probe: fixed cost of one kernel launch + completion wait on MI355X (what a tick pays
// before doing any work), measured with hipEvents and host wall clock.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>
#include <sched.h>
#include <sys/prctl.h>

__global__ void empty_k(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

int main() {
  int* d;
  hipMalloc(&d, 64);
  hipMemset(d, 0, 64);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {1, 256, 1024}) {
    double ev_us = 0, wall_us = 0, wall_poll = 0;
    const int N = 200;
    for (int i = 0; i < N + 10; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      hipEventRecord(e0, st);
      hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d);
      hipEventRecord(e1, st);
      hipStreamSynchronize(st);
      auto t1 = std::chrono::steady_clock::now();
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // poll-with-sleep variant (what HipEngine::wait_stream does)
      auto t2 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d);
      while (hipStreamQuery(st) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(15));
      auto t3 = std::chrono::steady_clock::now();
      if (i >= 10) {
        ev_us += ms * 1000.0;
        wall_us += std::chrono::duration<double, std::micro>(t1 - t0).count();
        wall_poll += std::chrono::duration<double, std::micro>(t3 - t2).count();
      }
    }
    printf("grid %4d: event-timed %.1f us, launch+sync wall %.1f us, launch+poll/sleep wall %.1f us\n", grid,
           ev_us / N, wall_us / N, wall_poll / N);
  }
  // completion-wait variants for a ~100 us kernel-free tick
  hipEvent_t eb;
  hipEventCreateWithFlags(&eb, hipEventBlockingSync | hipEventDisableTiming);
  auto run = [&](const char* name, auto&& wait) {
    double t = 0;
    const int N = 300;
    for (int i = 0; i < N + 10; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(empty_k, dim3(256), dim3(256), 0, st, d);
      wait();
      auto t1 = std::chrono::steady_clock::now();
      if (i >= 10) t += std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    printf("%-40s %.1f us\n", name, t / N);
  };
  run("poll + sleep_for(15us) default slack", [&] {
    while (hipStreamQuery(st) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(15));
  });
  run("poll + sched_yield", [&] {
    while (hipStreamQuery(st) == hipErrorNotReady) sched_yield();
  });
  run("blocking-sync event", [&] {
    hipEventRecord(eb, st);
    hipEventSynchronize(eb);
  });
  prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
  run("poll + sleep_for(15us) slack 1ns", [&] {
    while (hipStreamQuery(st) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(15));
  });
  run("poll + sleep_for(5us) slack 1ns", [&] {
    while (hipStreamQuery(st) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(5));
  });
  return 0;
}
