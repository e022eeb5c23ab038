"""Configuration layer (SURVEY §2.6 schema, §5.6 config system).

Keeps quorum's YAML schema and every ``.get(..., default)`` default bit-for-bit
(reference ``src/quorum/oai_proxy.py:40-63`` for the loader and default config,
``:1049-1075`` / ``:1166-1189`` for the per-strategy flag defaults, ``:772-825`` for the
aggregate block).  Additions, none of which change reference semantics:

* ``--config PATH`` / ``QMX_CONFIG`` override the file location;
* ``validate_config`` gives clear errors (opt-in; the loader keeps the silent
  default-config fallback of the reference, but logs it loudly);
* a separate ``runtime`` section holds MI355X knobs (device, tick, batch caps,
  placement) — see :class:`RuntimeConfig`.
"""
from __future__ import annotations

import copy
import logging
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional

import yaml

logger = logging.getLogger("quorum_amd.config")

DEFAULT_THINKING_TAGS: List[str] = ["think", "reason", "reasoning", "thought"]
DEFAULT_PROMPT_TEMPLATE = (
    "You have received the following responses regarding the user's query:\n\n"
    "{responses}\n\nProvide a concise synthesis of these responses."
)
DEFAULT_QUERY_FORMAT = "Original query: {query}\n\n"
DEFAULT_SOURCE_LABEL_FORMAT = "Response from {backend_name}:\n"
DEFAULT_INTERMEDIATE_SEPARATOR = "\n\n---\n\n"

# reference oai_proxy.py:54-63
DEFAULT_CONFIG: Dict[str, Any] = {
    "primary_backends": [
        {"name": "default", "url": "https://api.openai.com/v1", "model": ""}
    ],
    "settings": {"timeout": 60},
}

REPO_ROOT = Path(__file__).resolve().parent.parent.parent


def default_config_path() -> Path:
    env = os.environ.get("QMX_CONFIG")
    if env:
        return Path(env)
    return REPO_ROOT / "config.yaml"


def load_config(path: Optional[os.PathLike] = None) -> Dict[str, Any]:
    """Load the YAML config; on ANY error return the reference default config.

    Mirrors reference ``load_config`` (oai_proxy.py:40-63): ``yaml.safe_load`` of the
    file, silent fallback to a single OpenAI backend with ``timeout: 60``.
    """
    cfg_path = Path(path) if path is not None else default_config_path()
    try:
        text = cfg_path.read_text()
        cfg = yaml.safe_load(text)
        logger.info("loaded configuration from %s", cfg_path)
        return cfg
    except Exception as exc:  # noqa: BLE001 - reference behaviour: any error -> default
        logger.error("error loading %s (%s); using the default configuration", cfg_path, exc)
        return copy.deepcopy(DEFAULT_CONFIG)


class ConfigError(ValueError):
    pass


def validate_config(cfg: Dict[str, Any]) -> List[str]:
    """Strict validation (opt-in). Returns a list of warnings; raises ConfigError on errors."""
    warnings: List[str] = []
    if not isinstance(cfg, dict):
        raise ConfigError("config root must be a mapping")
    backends = cfg.get("primary_backends")
    if not isinstance(backends, list) or not backends:
        raise ConfigError("primary_backends must be a non-empty list")
    names = set()
    for i, b in enumerate(backends):
        if not isinstance(b, dict):
            raise ConfigError(f"primary_backends[{i}] must be a mapping")
        for key in ("name", "url", "model"):
            if key not in b:
                raise ConfigError(f"primary_backends[{i}] is missing '{key}'")
        if b["name"] in names:
            warnings.append(f"duplicate backend name {b['name']!r}")
        names.add(b["name"])
        if not b.get("url"):
            warnings.append(f"backend {b['name']!r} has no url and will be ignored")
    if not isinstance(cfg.get("settings"), dict):
        raise ConfigError("settings must be a mapping (reference crashes at import without it)")
    sel = strategy_name(cfg)
    if "strategy" in cfg and sel not in (cfg.get("strategy") or {}):
        warnings.append(f"selected strategy {sel!r} has no block under 'strategy'; defaults apply")
    agg = (cfg.get("strategy") or {}).get("aggregate") or {}
    sem = cfg.get("semantics", "reference")
    if sem not in SEMANTICS:
        raise ConfigError(f"semantics must be one of {SEMANTICS}, not {sem!r}")
    if sem == "reference":
        for unused in ("strip_intermediate_thinking", "hide_aggregator_thinking"):
            if unused in agg:
                warnings.append(f"strategy.aggregate.{unused} is accepted but, as in quorum, has no effect "
                                "(set semantics: documented to honour it)")
    else:
        src = agg.get("source_backends", "all")
        for n in ([src] if isinstance(src, str) and src != "all" else src if isinstance(src, list) else []):
            if n not in names:
                warnings.append(f"source_backends names {n!r}, which is not a primary backend")
    if agg.get("aggregator_backend") and agg["aggregator_backend"] not in names:
        warnings.append(f"aggregator_backend {agg['aggregator_backend']!r} is not a primary backend")
    return warnings


# ``semantics``: "reference" (default) reproduces quorum's code, including the flags its docs
# describe but its code ignores; "documented" honours those flags as docs/aggregate_behaviour.md
# describes them (SURVEY §2.8 "documented behaviour"): source_backends, strip_intermediate_thinking,
# hide_aggregator_thinking, backend-name source labels, and the non-stream
# suppress_individual_responses ("only the first response").
SEMANTICS = ("reference", "documented")


def documented(cfg: Dict[str, Any]) -> bool:
    return (cfg or {}).get("semantics", "reference") == "documented"


def strategy_name(cfg: Dict[str, Any]) -> str:
    return (cfg.get("iterations") or {}).get("aggregation", {}).get("strategy", "concatenate")


@dataclass
class StrategyFlags:
    """Per-request resolved strategy flags (reference oai_proxy.py:1049-1075)."""

    name: str = "concatenate"
    separator: str = "\n"
    hide_intermediate_think: bool = True
    hide_final_think: bool = False
    thinking_tags: List[str] = field(default_factory=lambda: list(DEFAULT_THINKING_TAGS))
    skip_final_aggregation: bool = False
    suppress_individual_responses: bool = False


@dataclass
class AggregateSettings:
    """``strategy.aggregate`` block (reference oai_proxy.py:772-825, 1205-1268).

    NOTE: like quorum, this block is consulted regardless of the selected
    strategy (oai_proxy.py:772/1205) — with an ``aggregator_backend`` set, even
    ``concatenate`` routes the final through the aggregator.
    """

    aggregator_backend: Optional[str] = None
    source_backends: Any = "all"  # computed-but-unused in quorum (oai_proxy.py:774-780)
    prompt_template: str = DEFAULT_PROMPT_TEMPLATE
    intermediate_separator: str = DEFAULT_INTERMEDIATE_SEPARATOR
    include_original_query: bool = True
    query_format: str = DEFAULT_QUERY_FORMAT
    include_source_names: bool = False
    source_label_format: str = DEFAULT_SOURCE_LABEL_FORMAT
    # honoured only with ``semantics: documented`` (see SEMANTICS above)
    documented: bool = False
    strip_intermediate_thinking: bool = False
    hide_aggregator_thinking: bool = False

    def sources(self) -> Optional[List[str]]:
        """Backend names whose texts feed the aggregator (documented mode); None = all."""
        if not self.documented or self.source_backends == "all" or self.source_backends is None:
            return None
        if isinstance(self.source_backends, str):
            return [self.source_backends]
        return [str(n) for n in self.source_backends]


def resolve_flags(cfg: Dict[str, Any], body: Optional[Dict[str, Any]] = None) -> StrategyFlags:
    name = strategy_name(cfg)
    block = (cfg.get("strategy") or {}).get(name, {}) or {}
    flags = StrategyFlags(
        name=name,
        separator=block.get("separator", "\n"),
        hide_intermediate_think=block.get("hide_intermediate_think", True),
        hide_final_think=block.get("hide_final_think", False),
        thinking_tags=list(block.get("thinking_tags", DEFAULT_THINKING_TAGS)),
        skip_final_aggregation=block.get("skip_final_aggregation", False),
        suppress_individual_responses=block.get("suppress_individual_responses", False),
    )
    if body is not None and isinstance(body, dict) and "suppress_individual_responses" in body:
        flags.suppress_individual_responses = body.get("suppress_individual_responses")
    return flags


def resolve_aggregate(cfg: Dict[str, Any]) -> AggregateSettings:
    block = (cfg.get("strategy") or {}).get("aggregate", {}) or {}
    template = block.get("prompt_template", DEFAULT_PROMPT_TEMPLATE)
    if "{intermediate_results}" in template:  # reference oai_proxy.py:806-809
        template = template.replace("{intermediate_results}", "{responses}")
    return AggregateSettings(
        aggregator_backend=block.get("aggregator_backend"),
        source_backends=block.get("source_backends", "all"),
        prompt_template=template,
        intermediate_separator=block.get("intermediate_separator", DEFAULT_INTERMEDIATE_SEPARATOR),
        include_original_query=block.get("include_original_query", True),
        query_format=block.get("query_format", DEFAULT_QUERY_FORMAT),
        include_source_names=block.get("include_source_names", False),
        source_label_format=block.get("source_label_format", DEFAULT_SOURCE_LABEL_FORMAT),
        documented=documented(cfg),
        strip_intermediate_thinking=bool(block.get("strip_intermediate_thinking", False)),
        hide_aggregator_thinking=bool(block.get("hide_aggregator_thinking", False)),
    )


def find_backend(cfg: Dict[str, Any], name: Optional[str]) -> Optional[Dict[str, Any]]:
    if not name:
        return None
    for b in cfg.get("primary_backends", []) or []:
        if b.get("name") == name:
            return b
    return None


def valid_backends(cfg: Dict[str, Any]) -> List[Dict[str, Any]]:
    return [b for b in cfg.get("primary_backends", []) if b.get("url")]


def is_parallel(cfg: Dict[str, Any], n_valid: int) -> bool:
    """reference oai_proxy.py:1043-1044."""
    return ("iterations" in cfg and "strategy" in cfg) and n_valid > 1


def request_timeout(cfg: Dict[str, Any]) -> float:
    return float((cfg.get("settings") or {}).get("timeout", 60))


@dataclass
class RuntimeConfig:
    """MI355X runtime knobs (``runtime:`` YAML section / env). Never changes semantics.

    engine:    "auto" (hip when a GPU is visible, else cpu) | "hip" | "cpu" | "python"
    device:    HIP device ordinal (default LOCAL_RANK)
    tile_bytes: per-stream input bytes per tick (LDS tile in the fused tick kernel)
    max_slots: concurrent upstream streams resident per rank
    content_cap: device-resident filtered-content bytes per stream slot
    placement: "local" (a session's backends run on the owner rank) | "spread" (EP analog)
    exchange:  spread transport: "auto" (rccl with a GPU engine, else tcp) | "rccl" | "tcp"
    exchange_round_us: pacing of the lock-step all-gather rounds while traffic flows
    exchange_timeout: a round slower than this = peer failure (fall back to local placement)
    exchange_eager_bytes: spread final texts up to this size ride the mesh right behind their
               deltas (eager); larger ones take a bulk round — rank-0 manifest, RCCL / socket
               transfer (rendezvous); 0 = every text takes a round — QMX_XCHG_EAGER_BYTES
    total_timeout: optional per-backend total deadline in seconds (None = quorum semantics)
    drain_timeout: SIGTERM grace period for in-flight sessions (rolling reload / shutdown)
    verify:    debug mode: a shadow CPU oracle engine checks every stream and final (QMX_VERIFY=1)
    shared_engine: "auto" (one engine per process shared by all io loops for hip, per-loop
               engines for cpu) | true | false (QMX_SHARED_ENGINE=0/1)
    tick_lanes: shared engine: tick threads with a kernel in flight each (own HIP stream and
               arenas, disjoint stream sets) — QMX_TICK_LANES
    tick_mode: hip engine: "loops" (every io loop owns an engine and posts its own ticks into
               one shared multi-door persistent grid, applying the results itself — no tick
               thread in between) | "lanes" (one shared engine ticked by `tick_lanes` threads)
               | "auto" (loops — spread placement included; lanes only with tick_mode "lanes", an
               explicit shared engine, or a grid that does not fit the GPU) — QMX_TICK_MODE
    log_content: allow prompts / per-backend answers in the ``aggregation`` log (off: user
               data; see utils/logging_setup.py) — QMX_LOG_CONTENT
    watch_config: the supervisor polls the config file and rolls a new worker generation in
               when its content changes (the reference's ``uvicorn --reload --reload-include
               "*.yaml"``, Makefile:4; here without dropping a request) — QMX_WATCH_CONFIG
    watch_interval: seconds between those polls
    read_pace_us: an io-loop pass that read trickling upstreams (short reads of responses still
               in progress: one SSE event per write, as LLM servers send tokens) lasts at least
               this long, so the events that arrive meanwhile share one receive per socket, one
               wait and one client send; whole-response reads never trigger it.  MI355X box,
               headline-shaped trickle: 33k -> 41k req/s and 192 -> 82 us proxy CPU per request at
               50 us, p50 TTFT +0.08 ms (profiles/r6/pacing).  0: off — QMX_READ_PACE_US
    light_host_sessions: the HIP engine's latency mode — a session opened on an io loop with no
               tick on the GPU, which has served at most this many sessions at a time lately,
               runs its streams on the host path (the byte-identical C++ engine, inline): p50
               TTFT 0.040 -> 0.018 ms at one connection, neutral at the headline's load
               (profiles/r6/lowload/light_host).  0: off; unset: QMX_LIGHT_HOST, which `serve`
               sets to 2 for its workers and bench.py to 0
    """

    engine: str = "auto"
    device: Optional[int] = None
    tile_bytes: int = 16384
    max_slots: int = 8192
    content_cap: int = 1 << 20
    placement: str = "local"
    exchange: str = "auto"
    exchange_round_us: int = 200
    exchange_timeout: float = 30.0
    exchange_eager_bytes: int = 4096
    total_timeout: Optional[float] = None
    drain_timeout: float = 10.0
    verify: bool = False
    shared_engine: Any = "auto"
    tick_lanes: int = 2
    tick_mode: str = "auto"
    log_content: bool = False
    watch_config: bool = False
    watch_interval: float = 1.0
    read_pace_us: int = 50
    light_host_sessions: Optional[int] = None

    @classmethod
    def from_config(cls, cfg: Dict[str, Any]) -> "RuntimeConfig":
        rt = dict((cfg or {}).get("runtime") or {})
        env_engine = os.environ.get("QMX_ENGINE")
        if env_engine:
            rt["engine"] = env_engine
        if os.environ.get("QMX_PLACEMENT"):
            rt["placement"] = os.environ["QMX_PLACEMENT"]
        if os.environ.get("QMX_VERIFY"):
            rt["verify"] = os.environ["QMX_VERIFY"] not in ("0", "", "false")
        if os.environ.get("QMX_SHARED_ENGINE"):
            rt["shared_engine"] = os.environ["QMX_SHARED_ENGINE"] not in ("0", "false")
        if os.environ.get("QMX_WATCH_CONFIG"):
            rt["watch_config"] = os.environ["QMX_WATCH_CONFIG"] not in ("0", "", "false")
        if os.environ.get("QMX_TICK_LANES"):
            rt["tick_lanes"] = int(os.environ["QMX_TICK_LANES"])
        if os.environ.get("QMX_TICK_MODE"):
            rt["tick_mode"] = os.environ["QMX_TICK_MODE"]
        if os.environ.get("QMX_READ_PACE_US"):
            rt["read_pace_us"] = int(os.environ["QMX_READ_PACE_US"])
        known = {k: v for k, v in rt.items() if k in cls.__dataclass_fields__}
        return cls(**known)
