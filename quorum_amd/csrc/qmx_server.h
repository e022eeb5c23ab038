// qmx_server.h — native data plane: epoll HTTP/1.1 proxy front-end + upstream client.
//
// One process per GPU; T io threads per process, each owning an SO_REUSEPORT listener, its
// client/upstream connections and keep-alive upstream pools.  Stream processing: for `hip`
// one shared engine per process (the GPU hub) whose tick lanes — threads, each with its own
// HIP stream and host-mapped arenas — keep up to `tick_lanes` fused tick kernels in flight
// over disjoint stream sets while the io loops keep reading sockets; for `cpu` one engine
// per io loop, ticked inline.  Semantics mirror the FastAPI
// conformance app (quorum_amd/server/app.py) and quorum's handler
// (src/quorum/oai_proxy.py:959-1408).
#pragma once
#include <netinet/in.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace qmx {

struct BackendCfg {
  std::string name, url, model;
  bool has_model_key = true;  // quorum indexes backend["model"] (KeyError → proxy_error)
  bool valid = false;         // url truthy
  std::string host, path;     // parsed http URL
  int port = 80;
  bool https = false;
  sockaddr_in addr{};
  bool resolved = false;
};

struct ServerCfg {
  std::string host = "127.0.0.1";
  int port = 8000;
  int threads = 2;
  // engine
  std::string engine = "cpu";
  int shared_engine = -1;  // one engine per process shared by all io loops (-1: auto = hip only)
  int tick_lanes = 2;      // shared engine: tick threads, each with its own HIP stream + arenas
  // hip: "loops" = every io loop owns an engine and posts its own ticks into one multi-door
  // persistent grid (HipGrid), "lanes" = the shared engine + tick-lane threads (GpuHub),
  // "auto" = loops (spread placement included); lanes only when asked (tick_mode "lanes",
  // shared_engine = 1) or when the grid does not fit the GPU
  std::string tick_mode = "auto";
  // read pacing: a loop pass that read trickling upstreams (short reads of responses in
  // progress) lasts at least this long, so events arriving meanwhile share receives, waits and
  // client sends (0: off; QMX_READ_PACE_US overrides)
  int read_pace_us = 50;
  // the HIP engine's latency mode: at most this many sessions per io loop lately, and no tick
  // on the GPU, and a new session's streams run on the host path (-1: QMX_LIGHT_HOST, else 0)
  int light_host = -1;
  int device = 0;
  int tile = 16384, max_slots = 4096, content_cap = 1 << 20;
  // config
  std::vector<BackendCfg> backends;  // all primary_backends (config order)
  bool has_iterations_and_strategy = false;
  double timeout = 60.0;
  double total_timeout = 0.0;  // 0 = none (quorum semantics)
  std::string separator = "\n";
  bool hide_intermediate = true, hide_final = false, skip_final = false, suppress = false;
  std::vector<std::string> tags;
  // strategy.aggregate (consulted whatever strategy is selected, as in quorum)
  std::string aggregator_name;  // empty = none
  std::string prompt_template, intermediate_separator, query_format, source_label_format;
  bool include_original_query = true, include_source_names = false;
  // semantics "documented" (utils/config.py SEMANTICS): the flags of the reference's
  // docs/aggregate_behaviour.md, which its code ignores — source_backends (sources_all false:
  // only `sources` feed the aggregator), strip_intermediate_thinking, hide_aggregator_thinking,
  // backend-name source labels, non-stream suppress = the first response
  bool documented = false, strip_intermediate = false, hide_aggregator_think = false, sources_all = true;
  std::vector<std::string> sources;
  std::string env_api_key;         // static OPENAI_API_KEY (tests; api_key_from_env = false)
  bool api_key_from_env = false;   // read OPENAI_API_KEY per request, as quorum (oai_proxy.py:981)
  // FastAPI's default documentation routes of the reference app (oai_proxy.py:70): the
  // documents are rendered once by the launcher from the conformance app; empty = 404
  std::string openapi_json, docs_html, redoc_html, oauth2_redirect_html;
  bool install_signals = true;
  // multi-rank: one process per GPU.  placement "local" = DP session sharding only;
  // "spread" = a session's backend streams run on ranks owner..owner+N-1 (qmx_exchange.h)
  int rank = 0, world = 1;
  std::string placement = "local";
  std::string xchg = "tcp";  // tcp | rccl
  std::string xchg_addr = "127.0.0.1";
  int xchg_port = 0;
  int xchg_bulk_port = 0;  // tcpbulk: rank r listens on xchg_bulk_port + r (0: xchg_port + world)
  std::string xchg_id_file;
  int xchg_round_us = 200;
  // spread: a final text up to this size rides the mesh right behind its deltas (eager: no
  // round, no rank-0 manifest — the MPI eager protocol); a larger one takes a bulk round
  // (rendezvous: manifest + RCCL / socket transfer).  0: every final text takes a round
  int xchg_eager_bytes = 4096;
  int xchg_links = -1;  // per-loop exchange links: 1 on, 0 off, -1 QMX_XCHG_LINKS (default on)
  double xchg_timeout = 30.0;
  // lifecycle: SIGTERM drains (no new connections; in-flight sessions finish, at most
  // drain_s seconds), SIGINT / stop_server() stop at once; ready_file is written once
  // every io loop is listening (supervisor rolling reloads)
  double drain_s = 10.0;
  std::string ready_file;
  // admin_port > 0: io loop 0 also listens here, without SO_REUSEPORT — a port that reaches
  // exactly this process (/metrics and /health of ONE rank; bench.py scrapes it per rank)
  int admin_port = 0;
  bool verify = false;  // shadow CPU oracle engine compares every stream + finalize result
  // https upstreams: CA bundle (httpx default: certifi) and peer verification
  std::string ca_file;
  bool tls_verify = true;
};

// Runs until SIGINT / stop_server(), or until drained after SIGTERM. Returns 0.
int run_server(const ServerCfg& cfg);
std::unordered_map<std::string, double> server_counters();
void stop_server();  // thread-safe; run_server returns within ~50 ms

}  // namespace qmx
