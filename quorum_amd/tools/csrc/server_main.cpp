// qmx_server — the native data plane as a standalone binary (no Python in the process).
//
//   qmx_server config.json          # the flat dict that quorum_amd.runtime.native_server
//                                   # .native_config() produces, serialised as JSON
//
// Used for the sanitizer build (qmx_server_asan: -fsanitize=address,undefined on host code)
// and for deployments that want one C++ process per GPU.  SIGTERM drains, SIGINT stops.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "qmx_json.h"
#include "qmx_server.h"

using namespace qmx;

namespace {

std::string gs(const JVal& d, const char* k, const std::string& dflt) {
  const JVal* v = d.get(k);
  return v && v->t == JVal::STR ? v->s : dflt;
}
double gd(const JVal& d, const char* k, double dflt) {
  const JVal* v = d.get(k);
  if (!v) return dflt;
  if (v->t == JVal::FLOAT) return v->d;
  if (v->t == JVal::INT) return atof(v->s.c_str());
  if (v->t == JVal::TRUE_) return 1;
  if (v->t == JVal::FALSE_) return 0;
  return dflt;
}
bool gb(const JVal& d, const char* k, bool dflt) { return gd(d, k, dflt ? 1 : 0) != 0; }
int gi(const JVal& d, const char* k, int dflt) { return (int)gd(d, k, dflt); }

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: qmx_server config.json\n");
    return 2;
  }
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string text = ss.str(), err;
  JVal d;
  if (!json_parse(text.data(), text.size(), d, &err) || d.t != JVal::OBJ) {
    fprintf(stderr, "qmx_server: bad config %s: %s\n", argv[1], err.c_str());
    return 2;
  }
  ServerCfg c;
  c.host = gs(d, "host", c.host);
  c.port = gi(d, "port", c.port);
  c.threads = gi(d, "threads", c.threads);
  c.engine = gs(d, "engine", c.engine);
  c.device = gi(d, "device", c.device);
  c.tile = gi(d, "tile", c.tile);
  c.max_slots = gi(d, "max_slots", c.max_slots);
  c.content_cap = gi(d, "content_cap", c.content_cap);
  c.has_iterations_and_strategy = gb(d, "has_iterations_and_strategy", false);
  c.timeout = gd(d, "timeout", c.timeout);
  c.total_timeout = gd(d, "total_timeout", c.total_timeout);
  c.separator = gs(d, "separator", c.separator);
  c.hide_intermediate = gb(d, "hide_intermediate", c.hide_intermediate);
  c.hide_final = gb(d, "hide_final", c.hide_final);
  c.skip_final = gb(d, "skip_final", c.skip_final);
  c.suppress = gb(d, "suppress", c.suppress);
  if (const JVal* t = d.get("tags"))
    for (auto& x : t->a) c.tags.push_back(x.s);
  c.aggregator_name = gs(d, "aggregator_name", "");
  c.prompt_template = gs(d, "prompt_template", "");
  c.intermediate_separator = gs(d, "intermediate_separator", "");
  c.query_format = gs(d, "query_format", "");
  c.source_label_format = gs(d, "source_label_format", "");
  c.include_original_query = gb(d, "include_original_query", true);
  c.include_source_names = gb(d, "include_source_names", false);
  c.documented = gb(d, "documented", false);
  c.strip_intermediate = gb(d, "strip_intermediate", false);
  c.hide_aggregator_think = gb(d, "hide_aggregator_think", false);
  c.sources_all = gb(d, "sources_all", true);
  if (const JVal* t = d.get("sources"))
    for (auto& x : t->a) c.sources.push_back(x.s);
  c.env_api_key = gs(d, "env_api_key", "");
  c.api_key_from_env = gb(d, "api_key_from_env", false);
  c.openapi_json = gs(d, "openapi_json", "");
  c.docs_html = gs(d, "docs_html", "");
  c.redoc_html = gs(d, "redoc_html", "");
  c.oauth2_redirect_html = gs(d, "oauth2_redirect_html", "");
  c.rank = gi(d, "rank", 0);
  c.world = gi(d, "world", 1);
  c.placement = gs(d, "placement", "local");
  c.xchg = gs(d, "xchg", "tcp");
  c.xchg_addr = gs(d, "xchg_addr", c.xchg_addr);
  c.xchg_port = gi(d, "xchg_port", 0);
  c.xchg_id_file = gs(d, "xchg_id_file", "");
  c.xchg_round_us = gi(d, "xchg_round_us", c.xchg_round_us);
  c.xchg_eager_bytes = gi(d, "xchg_eager_bytes", c.xchg_eager_bytes);
  c.xchg_timeout = gd(d, "xchg_timeout", c.xchg_timeout);
  c.drain_s = gd(d, "drain_s", c.drain_s);
  c.ready_file = gs(d, "ready_file", "");
  c.verify = gb(d, "verify", false);
  c.shared_engine = gi(d, "shared_engine", -1);
  c.tick_lanes = gi(d, "tick_lanes", c.tick_lanes);
  c.tick_mode = gs(d, "tick_mode", c.tick_mode);
  c.ca_file = gs(d, "ca_file", "");
  c.tls_verify = gb(d, "tls_verify", true);
  if (const JVal* bs = d.get("backends")) {
    for (auto& b : bs->a) {
      BackendCfg bc;
      bc.name = gs(b, "name", "");
      bc.url = gs(b, "url", "");
      bc.model = gs(b, "model", "");
      bc.has_model_key = gb(b, "has_model_key", true);
      bc.valid = gb(b, "valid", false);
      bc.host = gs(b, "host", "");
      bc.port = gi(b, "port", 80);
      bc.path = gs(b, "path", "");
      bc.https = gb(b, "https", false);
      c.backends.push_back(bc);
    }
  }
  return run_server(c);
}
