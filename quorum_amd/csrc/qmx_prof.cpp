// qmx_prof.cpp — see qmx_prof.h.
#include "qmx_prof.h"

#include <dlfcn.h>
#include <errno.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace qmx {
namespace {

constexpr int kDepth = 24;
constexpr size_t kMaxSamples = 1 << 17;  // ~65 s at the default 2 kHz of process CPU

struct Sample {
  int n;
  void* pc[kDepth];
};

Sample* g_ring = nullptr;
std::atomic<size_t> g_next{0};
std::atomic<bool> g_on{false};
std::string g_path;
int g_us = 500;

void on_prof(int, siginfo_t*, void*) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const int saved = errno;
  const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) g_ring[i].n = backtrace(g_ring[i].pc, kDepth);
  errno = saved;
}

}  // namespace

void prof_start() {
  const char* p = getenv("QMX_PROF");
  if (!p || !*p || g_ring) return;
  g_path = p;
  const size_t at = g_path.find("%p");  // per-process file: %p -> pid
  if (at != std::string::npos) g_path.replace(at, 2, std::to_string((long)getpid()));
  g_ring = static_cast<Sample*>(calloc(kMaxSamples, sizeof(Sample)));
  if (!g_ring) return;
  void* warm[4];
  backtrace(warm, 4);  // loads the unwinder outside the signal handler
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  if (const char* e = getenv("QMX_PROF_US")) g_us = std::max(50, atoi(e));
  itimerval tv{};
  tv.it_interval.tv_sec = g_us / 1000000;
  tv.it_interval.tv_usec = g_us % 1000000;
  tv.it_value = tv.it_interval;
  g_on.store(true);
  setitimer(ITIMER_PROF, &tv, nullptr);
}

void prof_thread() {
  // A process-wide ITIMER_PROF fires at most once per scheduler tick however many threads
  // burn CPU; a per-thread CPU-time timer per hot thread samples each of them fully.
  if (!g_on.load()) return;
  sigevent sev{};
  sev.sigev_notify = SIGEV_THREAD_ID;
  sev.sigev_signo = SIGPROF;
  sev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
  timer_t t;
  if (timer_create(CLOCK_THREAD_CPUTIME_ID, &sev, &t) != 0) return;
  itimerspec its{};
  its.it_interval.tv_sec = g_us / 1000000;
  its.it_interval.tv_nsec = (long)(g_us % 1000000) * 1000;
  its.it_value = its.it_interval;
  timer_settime(t, 0, &its, nullptr);  // lives until the thread exits (profiling only)
}

void prof_stop() {
  if (!g_ring || !g_on.exchange(false)) return;
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  FILE* f = fopen(g_path.c_str(), "w");
  if (!f) return;
  const size_t n = std::min(g_next.load(), kMaxSamples);
  fprintf(f, "# qmx cpu profile: %zu samples, frames innermost first (module+offset)\n", n);
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = g_ring[i];
    for (int k = 0; k < s.n; ++k) {
      Dl_info di;
      if (dladdr(s.pc[k], &di) && di.dli_fname) {
        // return addresses point after the call: -1 lands inside the calling instruction
        const uintptr_t off = (uintptr_t)s.pc[k] - (uintptr_t)di.dli_fbase - (k > 0 ? 1 : 0);
        fprintf(f, "%s%s+0x%lx", k ? ";" : "", di.dli_fname, (unsigned long)off);
      } else {
        fprintf(f, "%s?+0x%lx", k ? ";" : "", (unsigned long)(uintptr_t)s.pc[k]);
      }
    }
    fputc('\n', f);
  }
  fclose(f);
}

}  // namespace qmx
