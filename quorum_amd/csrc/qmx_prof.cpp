// qmx_prof.cpp — see qmx_prof.h.
#include "qmx_env.h"
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
#include <exception>
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

// ---- fatal-signal reporting ------------------------------------------------------------
constexpr int kFatal[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
struct sigaction g_prev[sizeof(kFatal) / sizeof(kFatal[0])];
std::atomic<bool> g_crash_on{false};
std::atomic<int> g_in_crash{0};

void put_str(const char* s) {
  ssize_t r = write(2, s, strlen(s));
  (void)r;
}
void put_num(long v) {
  char b[24];
  int i = 23;
  b[i] = 0;
  bool neg = v < 0;
  unsigned long u = neg ? (unsigned long)(-v) : (unsigned long)v;
  do {
    b[--i] = (char)('0' + u % 10);
    u /= 10;
  } while (u && i > 1);
  if (neg) b[--i] = '-';
  put_str(b + i);
}
void put_hex(uintptr_t v) {
  char b[20];
  int i = 19;
  b[i] = 0;
  do {
    b[--i] = "0123456789abcdef"[v & 15];
    v >>= 4;
  } while (v && i > 2);
  b[--i] = 'x';
  b[--i] = '0';
  put_str(b + i);
}

// frames as module+offset (dladdr reads already-loaded link maps; no allocation)
void dump_stack(int skip) {
  void* pc[48];
  const int n = backtrace(pc, 48);
  for (int k = skip; k < n; ++k) {
    Dl_info di;
    put_str("  #");
    put_num(k - skip);
    put_str(" ");
    if (dladdr(pc[k], &di) && di.dli_fname) {
      put_str(di.dli_fname);
      put_str("+");
      put_hex((uintptr_t)pc[k] - (uintptr_t)di.dli_fbase);
      if (di.dli_sname) {
        put_str(" (");
        put_str(di.dli_sname);
        put_str(")");
      }
    } else {
      put_hex((uintptr_t)pc[k]);
    }
    put_str("\n");
  }
}

void on_fatal(int sig, siginfo_t* si, void* uc) {
  if (g_in_crash.fetch_add(1) == 0) {
    put_str("qmx fatal: signal ");
    put_num(sig);
    put_str(" (");
    put_str(strsignal(sig));
    put_str(") in thread ");
    put_num((long)syscall(SYS_gettid));
    if (sig == SIGSEGV || sig == SIGBUS) {
      put_str(", fault address ");
      put_hex((uintptr_t)si->si_addr);
    }
    put_str(", pid ");
    put_num((long)getpid());
    put_str("\n");
    dump_stack(1);
  }
  // hand over: the handler installed before ours (Python faulthandler dumps the Python
  // stacks, then re-raises), else the default action (core / termination by the signal)
  for (size_t i = 0; i < sizeof(kFatal) / sizeof(kFatal[0]); ++i) {
    if (kFatal[i] != sig) continue;
    const struct sigaction& p = g_prev[i];
    if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
      sigaction(sig, &p, nullptr);
      p.sa_sigaction(sig, si, uc);
      return;
    }
    if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
      sigaction(sig, &p, nullptr);
      p.sa_handler(sig);
      return;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

void on_terminate() {
  put_str("qmx fatal: std::terminate");
  if (std::exception_ptr ep = std::current_exception()) {
    try {
      std::rethrow_exception(ep);
    } catch (const std::exception& e) {
      put_str(" (uncaught exception: ");
      put_str(e.what());
      put_str(")");
    } catch (...) {
      put_str(" (uncaught non-std exception)");
    }
  }
  put_str(" in thread ");
  put_num((long)syscall(SYS_gettid));
  put_str("\n");
  dump_stack(1);
  g_in_crash.fetch_add(1);  // the abort() below is reported already
  abort();
}

}  // namespace

void crash_thread() {
  // a fault on a blown stack needs a stack of its own to report from
  static thread_local bool done = false;
  if (done) return;
  done = true;
  const size_t sz = 64 * 1024;
  stack_t ss{};
  ss.ss_sp = malloc(sz);
  if (!ss.ss_sp) return;
  ss.ss_size = sz;
  sigaltstack(&ss, nullptr);
}

void crash_handler_install() {
  if (g_crash_on.exchange(true)) return;
  void* warm[4];
  backtrace(warm, 4);  // loads the unwinder outside the signal handler
  crash_thread();
  for (size_t i = 0; i < sizeof(kFatal) / sizeof(kFatal[0]); ++i) {
    struct sigaction sa {};
    sa.sa_sigaction = on_fatal;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kFatal[i], &sa, &g_prev[i]);
  }
  std::set_terminate(on_terminate);
}

void prof_start() {
  const char* p = env_get("QMX_PROF");
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
  if (const char* e = env_get("QMX_PROF_US")) g_us = std::max(50, atoi(e));
  // Only per-thread CPU-time timers (prof_thread, armed by every hot thread): a process-wide
  // ITIMER_PROF signal may be delivered to any thread, including one blocked in a join, and
  // would charge its stack with CPU it never used.  The kernel checks thread CPU timers at
  // the scheduler tick, so the effective rate is at most HZ per thread whatever g_us says.
  g_on.store(true);
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
