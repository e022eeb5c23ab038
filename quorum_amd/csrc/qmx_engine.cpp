// qmx_engine.cpp — host engine core + the sequential (oracle-equivalent) CPU algorithms.
#include "qmx_env.h"
#include "qmx_engine.h"

#include <cstdlib>
#include <ctime>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace qmx {

const char* kDeltaSuffix = "\"}, \"finish_reason\": null}]}\n\n";
const char* kFinalSuffix = "\"}, \"finish_reason\": \"stop\"}]}\n\n";

TagSet make_tagset(const std::vector<std::string>& tags) {
  TagSet ts;
  std::memset(&ts, 0, sizeof(ts));
  std::vector<std::string> seen;
  for (const auto& t0 : tags) {
    std::string t;
    for (char c : t0) t.push_back((char)lower_ascii((uint8_t)c));
    if (std::find(seen.begin(), seen.end(), t) != seen.end()) continue;
    // regex metacharacters change what quorum's alternation matches (oai_proxy.py:137,
    // 271-274); '<', '>' and '/' in a tag let one tag's pattern start inside another's, so
    // the token model (at most one pattern per '<') would not hold; non-ASCII would need
    // Unicode case folding.  Everything else is literal, exactly as in the regex.
    for (char ch : t) {
      const uint8_t c = (uint8_t)ch;
      const bool ok = c >= 0x20 && c < 0x7f && !std::strchr(".^$*+?{}[]\\|()<>/", (int)c);
      if (!ok) throw std::invalid_argument("tag needs regex semantics: " + t0);
    }
    if (t.empty() || (int)t.size() > kMaxTagLen) throw std::invalid_argument("unsupported tag length: " + t0);
    if (ts.n >= kMaxTags) throw std::invalid_argument("too many thinking tags");
    seen.push_back(t);
    ts.len[ts.n] = (int)t.size();
    std::memcpy(ts.name[ts.n], t.data(), t.size());
    ++ts.n;
  }
  if (ts.n == 0) throw std::invalid_argument("empty tag set");
  return ts;
}

// --------------------------------------------------------------------------------
// streaming filter: state (depth, tail); X = tail ++ text, token walk left to right
// --------------------------------------------------------------------------------
void filter_feed(const TagSet& ts, FilterState& fs, const uint8_t* text, size_t n, std::string& out) {
  std::string xs;
  xs.reserve(fs.tail_len + n);
  xs.append((const char*)fs.tail, fs.tail_len);
  xs.append((const char*)text, n);
  const uint8_t* x = (const uint8_t*)xs.data();
  int N = (int)xs.size();
  int i = 0;
  fs.tail_len = 0;
  while (true) {
    // next token at or after i (depth 0: opens only are tokens)
    int p = i, tok = 0, L = 0;
    for (; p < N; ++p) {
      if (x[p] != '<') continue;
      tok = match_at(x, N, p, ts, &L);
      if (tok > 0 || (tok < 0 && fs.depth > 0)) break;
      tok = 0;
    }
    if (p < N) {
      if (fs.depth == 0) {
        out.append((const char*)x + i, p - i);
        fs.depth = 1;
      } else {
        fs.depth = tok > 0 ? fs.depth + 1 : std::max(fs.depth - 1, 0);
      }
      i = p + L;
      continue;
    }
    // no more tokens: hold back a trailing partial tag from the LAST '<'
    int q = N - 1;
    while (q >= i && x[q] != '<') --q;
    bool hold = q >= i && pattern_prefix(x, q, N, ts, fs.depth == 0);
    int cut = hold ? q : N;
    if (fs.depth == 0) out.append((const char*)x + i, cut - i);
    if (hold) {
      fs.tail_len = N - q;
      std::memcpy(fs.tail, x + q, fs.tail_len);
    }
    return;
  }
}

// --------------------------------------------------------------------------------
// final strip: tokens, per-tag next-close links, leftmost-first walk, Unicode strip
// --------------------------------------------------------------------------------
std::string strip_final(const TagSet& ts, const uint8_t* x, size_t n) {
  struct Tok { int pos, len, id; };
  std::vector<Tok> toks;
  for (int p = 0; p < (int)n; ++p) {
    if (x[p] != '<') continue;
    int L = 0;
    int id = match_at(x, (int)n, p, ts, &L);
    if (id != 0) toks.push_back({p, L, id});
  }
  std::vector<int> next_close(toks.size(), -1);
  int last[kMaxTags];
  for (int t = 0; t < kMaxTags; ++t) last[t] = -1;
  for (int k = (int)toks.size() - 1; k >= 0; --k) {
    int id = toks[k].id;
    if (id > 0) next_close[k] = last[id - 1];
    else last[-id - 1] = k;
  }
  std::string out;
  out.reserve(n);
  int i = 0;
  for (int k = 0; k < (int)toks.size(); ++k) {
    if (toks[k].id <= 0 || toks[k].pos < i) continue;
    int j = next_close[k];
    if (j < 0) continue;
    out.append((const char*)x + i, toks[k].pos - i);
    i = toks[j].pos + toks[j].len;
    k = j;
  }
  out.append((const char*)x + i, n - i);
  int a = 0, b = (int)out.size();
  ustrip((const uint8_t*)out.data(), &a, &b);
  return out.substr(a, b - a);
}

// --------------------------------------------------------------------------------
// SSE encoding
// --------------------------------------------------------------------------------
size_t escaped_size(const uint8_t* y, size_t n) {
  size_t s = 0;
  for (size_t p = 0; p < n;) {
    uint32_t cp;
    p += wtf8_decode(y, (int)p, (int)n, &cp);
    s += escaped_len_cp(cp);
  }
  return s;
}
void escape_append(const uint8_t* y, size_t n, std::string& out) {
  uint8_t buf[12];
  for (size_t p = 0; p < n;) {
    uint32_t cp;
    p += wtf8_decode(y, (int)p, (int)n, &cp);
    int k = escape_cp(cp, buf);
    out.append((const char*)buf, k);
  }
}
static void delta_prefix_append(int index, int64_t created, std::string& out) {
  char b[224];
  const int n = snprintf(b, sizeof(b),
                         "data: {\"id\": \"chatcmpl-parallel-%d\", \"object\": \"chat.completion.chunk\", "
                         "\"created\": %lld, \"model\": \"parallel-proxy\", \"choices\": [{\"index\": 0, "
                         "\"delta\": {\"content\": \"",
                         index, (long long)created);
  out.append(b, (size_t)n);
}
std::string delta_prefix(int index, int64_t created) {
  std::string s;
  delta_prefix_append(index, created, s);
  return s;
}
std::string final_prefix(int64_t created) {
  return "data: {\"id\": \"chatcmpl-parallel-final\", \"object\": \"chat.completion.chunk\", \"created\": " +
         std::to_string(created) +
         ", \"model\": \"parallel-proxy\", \"choices\": [{\"index\": 0, \"delta\": {\"content\": \"";
}

// --------------------------------------------------------------------------------
// per-stream processing (sequential)
// --------------------------------------------------------------------------------
// Is x[a:b) a complete JSON string body (valid escapes, no control characters, no unescaped
// quote, strict UTF-8)?  The template fast path of the CPU engine (the HIP kernel's
// wave_str_body, sequentially).
static bool str_body_ok(const uint8_t* x, int a, int b) {
  for (int p = a; p < b; ++p) {
    const uint8_t c = x[p];
    if (c == '"' || c < 0x20) return false;
    if (c == '\\') {
      if (++p >= b) return false;
      const uint8_t d = x[p];
      if (d == 'u') {
        if (p + 4 >= b) return false;
        for (int k = 1; k <= 4; ++k)
          if (hexv(x[p + k]) < 0) return false;
        p += 4;
      } else if (!(d == '"' || d == '\\' || d == '/' || d == 'b' || d == 'f' || d == 'n' || d == 'r' || d == 't')) {
        return false;
      }
    }
  }
  return utf8_valid(x, a, b);
}

static void handle_event(const TagSet& ts, SlotCore& s, const uint8_t* e, int m, int64_t created,
                         std::string& out, std::string& scratch) {
  EvResult r;
  const int tp = (int)s.tpl_pre.size(), tsz = (int)s.tpl_suf.size();
  if (tp > 0 && m >= tp + tsz && std::memcmp(e, s.tpl_pre.data(), tp) == 0 &&
      std::memcmp(e + m - tsz, s.tpl_suf.data(), tsz) == 0 && str_body_ok(e, tp, m - tsz)) {
    r.kind = EV_CONTENT;  // same shape as this stream's last parsed content event
    r.str_a = tp;
    r.str_b = m - tsz;
  } else {
    r = classify_event(e, m);
    if (r.kind == EV_CONTENT && r.str_a <= 256 && m - r.str_b <= 64) {
      s.tpl_pre.assign((const char*)e, r.str_a);
      s.tpl_suf.assign((const char*)e + r.str_b, m - r.str_b);
    }
  }
  if (r.kind == EV_SKIP) return;
  if (r.kind == EV_ABORT) {
    s.aborted = true;
    return;
  }
  const int dl = json_unescape(e, r.str_a, r.str_b, nullptr);
  thread_local std::string c;  // unescaped content (reused: no allocation per event)
  c.resize((size_t)dl);
  json_unescape(e, r.str_a, r.str_b, (uint8_t*)&c[0]);
  scratch.clear();
  if (s.filter) filter_feed(ts, s.fs, (const uint8_t*)c.data(), c.size(), scratch);
  else scratch.assign(c);
  s.content += scratch;
  if (!scratch.empty() && s.emit) {
    delta_prefix_append(s.index, created, out);
    escape_append((const uint8_t*)scratch.data(), scratch.size(), out);
    out += kDeltaSuffix;
  }
}

void process_slot(const TagSet& ts, SlotCore& s, const uint8_t* data, size_t n, bool eof, int64_t created,
                  std::string& out) {
  if (s.aborted || s.done) return;
  s.carry.append((const char*)data, n);
  const uint8_t* x = (const uint8_t*)s.carry.data();
  int N = (int)s.carry.size();
  int pos = 0;
  if (!s.started) {
    while (pos < N) {
      int w = ws_at(x, pos, N);
      if (w <= 0) break;
      pos += w;
    }
    bool undecided = pos < N && ws_at(x, pos, N) < 0;
    if (pos >= N || (undecided && !eof)) {
      s.carry.erase(0, pos);
      if (eof) s.done = true;
      return;
    }
    s.started = true;
  }
  thread_local std::string scratch;
  int from = pos;  // no separator starts before `from` (memchr for '\n', then check the next byte)
  while (!s.aborted) {
    const void* nl = from < N ? memchr(x + from, '\n', (size_t)(N - from)) : nullptr;
    if (!nl) break;
    const int j = (int)((const uint8_t*)nl - x);
    if (j + 1 >= N) break;
    if (x[j + 1] != '\n') {
      from = j + 1;
      continue;
    }
    handle_event(ts, s, x + pos, j - pos, created, out, scratch);  // leftmost separator
    pos = from = j + 2;
  }
  if (s.aborted) {
    s.carry.clear();
    return;
  }
  if (eof) {
    if (pos < N) handle_event(ts, s, x + pos, N - pos, created, out, scratch);
    s.carry.clear();
    if (!s.aborted) s.done = true;
    return;
  }
  s.carry.erase(0, pos);
}

void finalize_texts(const TagSet& ts, const std::vector<std::string>& texts, const FinalizeReq& r,
                    FinalizeRes& out) {
  out.id = r.id;
  std::vector<std::string> kept;
  for (const auto& t : texts) {
    if (t.empty()) continue;
    kept.push_back(r.strip ? strip_final(ts, (const uint8_t*)t.data(), t.size()) : t);
  }
  if (r.texts) {
    out.kind = 2;
    out.texts = std::move(kept);
    return;
  }
  if (kept.empty()) {
    out.kind = 0;
    return;
  }
  std::string joined;
  for (size_t i = 0; i < kept.size(); ++i) {
    if (i) joined += r.joiner;
    joined += kept[i];
  }
  out.kind = 1;
  out.event = final_prefix(r.created);
  escape_append((const uint8_t*)joined.data(), joined.size(), out.event);
  out.event += kFinalSuffix;
}

// --------------------------------------------------------------------------------
// HostEngine
// --------------------------------------------------------------------------------
static double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

HostEngine::HostEngine(const std::vector<std::string>& tags) : ts_(make_tagset(tags)) {
  if (const char* pe = env_get("QMX_PIPELINE")) pipeline_ = atoi(pe) != 0;
}

int HostEngine::open(int index, bool filter, bool emit, uint32_t* gen) {
  std::lock_guard<std::mutex> g(mu_);
  int slot;
  if (!free_.empty()) {
    slot = free_.back();
    free_.pop_back();
  } else {
    slot = (int)meta_.size();
    meta_.emplace_back();
    core_.emplace_back();
  }
  open_reserved(slot, index, filter, emit, gen);
  return slot;
}

void HostEngine::reserve(int k, std::vector<int>& out) {
  std::lock_guard<std::mutex> g(mu_);
  for (int i = 0; i < k; ++i) {
    if (!free_.empty()) {
      out.push_back(free_.back());
      free_.pop_back();
    } else {
      out.push_back((int)meta_.size());
      meta_.emplace_back();
      core_.emplace_back();
    }
  }
}

void HostEngine::open_reserved(int slot, int index, bool filter, bool emit, uint32_t* gen) {
  // reset in place: a reused slot keeps its (small) buffers, so a new session costs no
  // allocation under the engine lock
  auto recycle = [](std::string& x) {
    if (x.capacity() > (64u << 10)) std::string().swap(x);
    else x.clear();
  };
  Meta& m = meta_[slot];
  m.gen += 1;
  m.live = true;
  m.dirty = m.eof = m.closed = m.busy = false;
  m.fresh = true;
  recycle(m.incoming);
  if (gen) *gen = m.gen;
  SlotCore& c = core_[slot];
  c.filter = filter;
  c.emit = emit;
  c.started = c.aborted = c.done = false;
  c.index = index;
  recycle(c.carry);
  c.fs = FilterState();
  recycle(c.content);
  recycle(c.tpl_pre);
  recycle(c.tpl_suf);
}

void HostEngine::feed(int slot, const std::string& data) {
  std::lock_guard<std::mutex> g(mu_);
  feed_locked(slot, data);
}

void HostEngine::finish(int slot) {
  std::lock_guard<std::mutex> g(mu_);
  finish_locked(slot);
}

void HostEngine::release(int slot) {
  std::lock_guard<std::mutex> g(mu_);
  release_locked(slot);
}

void HostEngine::apply_ops(std::vector<EngineOp>& ops, bool move_data) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& op : ops) {
    if (op.kind == EngineOp::FEED) {
      if (move_data) feed_locked_move(op.slot, op.data);
      else feed_locked(op.slot, op.data);
    }
    else if (op.kind == EngineOp::FINISH) finish_locked(op.slot);
    else release_locked(op.slot);
  }
}

void HostEngine::feed_locked(int slot, const std::string& data) {
  if (slot < 0 || slot >= (int)meta_.size() || !meta_[slot].live) return;
  Meta& m = meta_[slot];
  m.incoming += data;
  bytes_in_ += data.size();
  if (!m.dirty) {
    m.dirty = true;
    m.t_dirty = mono_s();
    dirty_.push_back(slot);
  }
}

// Same as feed_locked, but an empty backlog takes the payload's buffer instead of a copy
// (the common case: the previous tick consumed everything), shortening the lock hold.
void HostEngine::feed_locked_move(int slot, std::string& data) {
  if (slot < 0 || slot >= (int)meta_.size() || !meta_[slot].live) return;
  if (!meta_[slot].incoming.empty()) return feed_locked(slot, data);
  bytes_in_ += data.size();
  meta_[slot].incoming.swap(data);
  Meta& m = meta_[slot];
  if (!m.dirty) {
    m.dirty = true;
    m.t_dirty = mono_s();
    dirty_.push_back(slot);
  }
}

void HostEngine::finish_locked(int slot) {
  if (slot < 0 || slot >= (int)meta_.size() || !meta_[slot].live) return;
  Meta& m = meta_[slot];
  m.eof = true;
  if (!m.dirty) {
    m.dirty = true;
    m.t_dirty = mono_s();
    dirty_.push_back(slot);
  }
}

void HostEngine::release_locked(int slot) {
  if (slot < 0 || slot >= (int)meta_.size() || !meta_[slot].live) return;
  meta_[slot].live = false;
  meta_[slot].incoming.clear();
  pending_free_.push_back(slot);
}

int HostEngine::submit_finalize(const std::vector<int>& slots, bool strip, bool texts, const std::string& joiner,
                                int64_t created) {
  std::lock_guard<std::mutex> g(mu_);
  FinalizeReq r{++next_fid_, slots, strip, texts, joiner, created};
  fin_.push_back(std::move(r));
  return next_fid_;
}

bool HostEngine::has_work() {
  std::lock_guard<std::mutex> g(mu_);
  if (!fin_.empty()) return true;
  for (int s : dirty_)
    if (!meta_[s].busy) return true;
  return false;
}

bool HostEngine::pending(int slot) {
  std::lock_guard<std::mutex> g(mu_);
  if (slot < 0 || slot >= (int)meta_.size()) return false;
  const Meta& m = meta_[slot];
  return m.live && (m.dirty || m.busy || !m.incoming.empty());
}

bool HostEngine::job_take(Job& j, bool allow_fin) {
  j.work.clear();
  j.fin.clear();
  thread_local std::vector<int> keep;
  keep.clear();
  std::lock_guard<std::mutex> g(mu_);
  for (int s : pending_free_) {
    if (meta_[s].busy) {  // still in flight on another lane: free it once settled
      keep.push_back(s);
      continue;
    }
    on_free(s);
    free_.push_back(s);
  }
  pending_free_.swap(keep);
  keep.clear();
  j.work.reserve(dirty_.size());
  double now = 0;
  for (int s : dirty_) {
    Meta& m = meta_[s];
    if (m.busy && m.live) {  // this stream's previous tick is not settled: next time
      keep.push_back(s);
      continue;
    }
    m.dirty = false;
    if (!m.live) continue;
    if (m.t_dirty > 0) {
      if (now == 0) now = mono_s();
      take_wait_s_ += now - m.t_dirty;
      ++takes_;
    }
    Work w{s, std::string(), m.eof, m.fresh};
    w.data.swap(m.incoming);
    m.fresh = false;
    m.busy = true;
    j.work.push_back(std::move(w));
  }
  dirty_.swap(keep);
  if (allow_fin) j.fin.swap(fin_);
  if (!j.work.empty() || !j.fin.empty()) ++ticks_;
  return !j.work.empty() || !j.fin.empty();
}

void HostEngine::job_finish(Job& j, std::vector<SlotResult>& results, std::vector<int>& taken) {
  size_t out = 0;
  for (auto& r : results) out += r.size();
  for (auto& w : j.work) taken.push_back(w.slot);
  std::lock_guard<std::mutex> g(mu_);
  bytes_out_ += out;
  // a taken slot stays busy until settled, so it cannot be re-opened meanwhile: its
  // generation is the one the results belong to
  for (auto& r : results) r.gen = meta_[r.slot].gen;
}

bool HostEngine::tick(int64_t created, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane,
                      std::vector<int>* taken) {
  // per-thread scratch reused from tick to tick (a tick thread drives one lane)
  thread_local Job j;
  thread_local std::vector<int> slots;
  slots.clear();
  if (!job_take(j, true)) return false;
  run_tick(j.work, j.fin, created, results, fres, lane);
  std::vector<int>& tk = taken ? *taken : slots;
  job_finish(j, results, tk);
  if (!taken) settle(slots);
  return true;
}

void HostEngine::settle(const std::vector<int>& taken) {
  std::lock_guard<std::mutex> g(mu_);
  for (int s : taken) meta_[s].busy = false;
}

std::string HostEngine::text(int slot) {
  if (slot < 0 || slot >= (int)nslots()) return std::string();
  const SlotCore& c = core_[slot];
  return c.aborted ? std::string() : c.content;
}

size_t HostEngine::content_size(int slot) {
  if (slot < 0 || slot >= (int)nslots()) return 0;
  return core_[slot].content.size();
}

void HostEngine::set_remote_content(int slot, const std::string* bytes, size_t len, bool /*host_copied*/) {
  if (slot < 0 || slot >= (int)nslots()) return;
  core_[slot].content = bytes ? *bytes : std::string(len, '\0');
}

std::unordered_map<std::string, double> HostEngine::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return {{"ticks", (double)ticks_}, {"bytes_in", (double)bytes_in_}, {"bytes_out", (double)bytes_out_},
          {"takes", (double)takes_}, {"take_wait_us", take_wait_s_ * 1e6},
          {"slots", (double)meta_.size()}, {"free", (double)free_.size()}};
}

// --------------------------------------------------------------------------------
// CpuEngine
// --------------------------------------------------------------------------------
void CpuEngine::run_tick(std::vector<Work>& work, std::vector<FinalizeReq>& fin, int64_t created,
                         std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int /*lane*/) {
  for (auto& w : work) {
    SlotCore& c = core_[w.slot];
    bool was_closed = c.done || c.aborted;
    std::string out;
    process_slot(ts_, c, (const uint8_t*)w.data.data(), w.data.size(), w.eof, created, out);
    int flags = (c.done ? RF_DONE : 0) | (c.aborted ? RF_ABORTED : 0);
    if (!out.empty() || (flags && !was_closed)) results.push_back({w.slot, std::move(out), flags});
  }
  for (auto& r : fin) {
    std::vector<std::string> texts;
    for (int s : r.slots) texts.push_back(text(s));
    FinalizeRes fr;
    finalize_texts(ts_, texts, r, fr);
    fres.push_back(std::move(fr));
  }
}

}  // namespace qmx

namespace qmx {

struct AsyncCpuEngine::Done {
  std::vector<SlotResult> results;
  std::vector<FinalizeRes> fres;
  std::atomic<bool> ready{false};
};

AsyncCpuEngine::AsyncCpuEngine(const std::vector<std::string>& tags) : CpuEngine(tags) {
  th_ = std::thread([this] { run(); });
}

AsyncCpuEngine::~AsyncCpuEngine() {
  {
    std::lock_guard<std::mutex> g(qmu_);
    stop_ = true;
  }
  qcv_.notify_all();
  if (th_.joinable()) th_.join();
}

void AsyncCpuEngine::job_post(Job& j) {
  auto d = std::make_shared<Done>();
  j.impl = d;
  inflight_.fetch_add(1, std::memory_order_acq_rel);
  {
    std::lock_guard<std::mutex> g(qmu_);
    q_.push_back(&j);
  }
  qcv_.notify_one();
}

void AsyncCpuEngine::run() {
  for (;;) {
    Job* j = nullptr;
    {
      std::unique_lock<std::mutex> lk(qmu_);
      qcv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stopping with nothing queued
      j = q_.front();
      q_.erase(q_.begin());
    }
    auto d = std::static_pointer_cast<Done>(j->impl);
    run_tick(j->work, j->fin, j->created, d->results, d->fres, 0);
    d->ready.store(true, std::memory_order_release);
  }
}

bool AsyncCpuEngine::job_ready(Job& j, double* expect_us) {
  if (expect_us) *expect_us = 5.0;
  auto d = std::static_pointer_cast<Done>(j.impl);
  return !d || d->ready.load(std::memory_order_acquire);
}

void AsyncCpuEngine::job_complete(Job& j, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) {
  auto d = std::static_pointer_cast<Done>(j.impl);
  if (!d) return;  // never posted
  for (auto& r : d->results) results.push_back(std::move(r));
  for (auto& f : d->fres) fres.push_back(std::move(f));
  j.impl.reset();
  inflight_.fetch_sub(1, std::memory_order_acq_rel);
}

}  // namespace qmx
