// qmx_env.h — environment reads that are safe on any thread.
//
// glibc's getenv walks `environ` with no lock; a concurrent setenv / putenv (the GPU runtime
// and other libraries write the environment while they initialise on their own threads, and
// in-process tests change it with monkeypatch) can reallocate that array under the walk.  A
// round-2 rehearsal lost a whole rank to exactly that: a tick lane's per-tick
// getenv("QMX_STAGE_TIMING") faulted inside getenv, the proxy process died, its peers marked
// it down and failed its remote streams (README "spread delta loss").
//
// Every read goes through a snapshot instead.  env_refresh() copies `environ` once — called
// on the main thread before a server / engine starts its threads (run_server, the bindings'
// engine constructors) — and env_get() only ever reads a published snapshot.  Old snapshots
// are kept alive (a refresh per server start), so a returned pointer stays valid.
#pragma once
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include <unistd.h>  // environ

namespace qmx {

using EnvMap = std::unordered_map<std::string, std::string>;

inline std::shared_ptr<const EnvMap>& env_slot() {
  static std::shared_ptr<const EnvMap> s;
  return s;
}
inline std::mutex& env_mu() {
  static std::mutex m;
  return m;
}

// Main thread, before the threads that read the environment start.
inline void env_refresh() {
  auto m = std::make_shared<EnvMap>();
  for (char** e = environ; e && *e; ++e) {
    const char* eq = std::strchr(*e, '=');
    if (eq) (*m)[std::string(*e, (size_t)(eq - *e))] = std::string(eq + 1);
  }
  std::lock_guard<std::mutex> g(env_mu());
  static std::vector<std::shared_ptr<const EnvMap>> keep;  // pointers handed out stay valid
  keep.push_back(m);
  std::atomic_store(&env_slot(), std::shared_ptr<const EnvMap>(m));
}

// The value of `name` in the last snapshot (nullptr: unset).  Never touches `environ` after
// the first snapshot.
inline const char* env_get(const char* name) {
  std::shared_ptr<const EnvMap> m = std::atomic_load(&env_slot());
  if (!m) {
    env_refresh();
    m = std::atomic_load(&env_slot());
  }
  auto it = m->find(name);
  return it == m->end() ? nullptr : it->second.c_str();
}

}  // namespace qmx
