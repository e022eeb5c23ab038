// qmx_prof.h — in-process CPU sampling profiler for the native data plane.
//
// QMX_PROF=<path> (%p = pid): SIGPROF every QMX_PROF_US (default 500) microseconds of each hot
// thread's own CPU time (a CLOCK_THREAD_CPUTIME_ID timer per thread that calls prof_thread();
// the kernel checks them at the scheduler tick, so at most HZ samples per thread per second);
// the handler records the interrupted thread's call stack into a preallocated ring
// (async-signal-safe: no allocation, one atomic slot claim).  prof_stop() writes one line per sample, frames as
// "module+0xoffset", for offline symbolisation (tools/cpuprof.py → llvm-symbolizer).
// A syscall shows up as its libc wrapper frame (the signal lands on the return to user
// space), so the profile splits the proxy's CPU into socket I/O, epoll, locking, HTTP /
// JSON handling and engine host work.  Not for production.
#pragma once

namespace qmx {

void prof_start();   // no-op unless QMX_PROF is set (idempotent)
void prof_thread();  // add a per-thread CPU-time sampler for the calling thread (if on)
void prof_stop();   // stop sampling, write the profile

// Fatal-signal reporting (SIGSEGV / SIGBUS / SIGFPE / SIGILL / SIGABRT and std::terminate):
// writes "qmx fatal: <signal> in thread <tid>" plus the faulting thread's backtrace
// (module+offset frames, symbolise with tools/cpuprof.py or llvm-symbolizer) to stderr on
// an alternate signal stack, then hands the signal to the previously installed handler
// (Python's faulthandler in a worker process) or the default action, so the exit status
// still reports the signal.  Idempotent; installs an alternate stack for the caller only
// (crash_thread() adds one per thread).
void crash_handler_install();
void crash_thread();

}  // namespace qmx
