"""Launch the native C++ data plane (quorum_amd/csrc/qmx_server.cpp) from a YAML config.

The YAML is resolved with the same helpers the FastAPI app uses (``quorum_amd.utils.config``)
so both front-ends share one definition of every default; the C++ server receives a flat,
fully-resolved dict.  Reference semantics: ``src/quorum/oai_proxy.py:959-1408``.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional
from urllib.parse import urlsplit

from ..utils.config import (RuntimeConfig, is_parallel, load_config, request_timeout, resolve_aggregate,
                            resolve_flags)


class NativeUnsupported(RuntimeError):
    pass


def native_config(cfg: Dict[str, Any], host: str, port: int, engine: str, device: Optional[int],
                  threads: int) -> Dict[str, Any]:
    if not isinstance(cfg, dict) or "primary_backends" not in cfg or not isinstance(cfg.get("settings"), dict):
        raise NativeUnsupported("config lacks primary_backends/settings (quorum would crash at import)")
    flags = resolve_flags(cfg)
    agg = resolve_aggregate(cfg)
    rt = RuntimeConfig.from_config(cfg)
    backends = []
    for b in cfg.get("primary_backends") or []:
        url = b.get("url") or ""
        parts = urlsplit(url) if url else None
        https = bool(parts and parts.scheme == "https")
        if parts and parts.scheme not in ("http", "https"):
            raise NativeUnsupported(f"backend {b.get('name')!r}: unsupported URL {url!r}")
        model = b.get("model", "")
        backends.append({
            "name": str(b.get("name", "")), "url": url, "model": "" if model is None else str(model),
            "has_model_key": "model" in b, "valid": bool(url), "https": https,
            "host": parts.hostname if parts else "",
            "port": (parts.port or (443 if https else 80)) if parts else 80,
            "path": (parts.path.rstrip("/") if parts else ""),
        })
    tags = [str(t) for t in flags.thinking_tags]
    from ..ops.engine import native_tag_ok

    if not native_tag_ok(tags):
        raise NativeUnsupported(f"thinking_tags {tags!r} need regex semantics: run with --impl python")
    if engine == "auto":
        from ..ops import native
        engine = "hip" if native.gpu_available() else "cpu"
    return {
        "host": host, "port": port, "threads": threads, "engine": engine,
        "device": int(device if device is not None else os.environ.get("LOCAL_RANK", "0")),
        "tile": rt.tile_bytes, "max_slots": rt.max_slots, "content_cap": rt.content_cap,
        "has_iterations_and_strategy": "iterations" in cfg and "strategy" in cfg,
        "timeout": request_timeout(cfg), "total_timeout": float(rt.total_timeout or 0.0),
        "separator": str(flags.separator), "hide_intermediate": bool(flags.hide_intermediate_think),
        "hide_final": bool(flags.hide_final_think), "skip_final": bool(flags.skip_final_aggregation),
        "suppress": bool(flags.suppress_individual_responses), "tags": tags,
        "aggregator_name": str(agg.aggregator_backend or ""), "prompt_template": str(agg.prompt_template),
        "intermediate_separator": str(agg.intermediate_separator), "query_format": str(agg.query_format),
        "source_label_format": str(agg.source_label_format),
        "include_original_query": bool(agg.include_original_query),
        "include_source_names": bool(agg.include_source_names),
        "documented": bool(agg.documented), "strip_intermediate": bool(agg.strip_intermediate_thinking),
        "hide_aggregator_think": bool(agg.hide_aggregator_thinking),
        "sources_all": agg.sources() is None, "sources": list(agg.sources() or []),
        "env_api_key": "", "api_key_from_env": True,  # per request, as quorum (oai_proxy.py:981)
        "backends": backends,
        "drain_s": float(rt.drain_timeout), "verify": bool(rt.verify),
        "shared_engine": -1 if rt.shared_engine in ("auto", None) else int(bool(rt.shared_engine)),
        "tick_lanes": int(rt.tick_lanes),
        "tick_mode": str(rt.tick_mode or "auto"),
        "read_pace_us": int(rt.read_pace_us),
        "light_host": -1 if rt.light_host_sessions is None else int(rt.light_host_sessions),
        "ca_file": _ca_bundle(), "tls_verify": os.environ.get("QMX_TLS_VERIFY", "1") not in ("0", "false"),
        "ready_file": (os.environ["QMX_READY_FILE"] + f".{os.getpid()}") if os.environ.get("QMX_READY_FILE") else "",
        # QMX_ADMIN_PORT: this process's own /metrics + /health port (not SO_REUSEPORT-shared)
        "admin_port": int(os.environ.get("QMX_ADMIN_PORT", "0")),
        **cluster_config(rt, port, engine),
        **doc_routes(cfg),
    }


def doc_routes(cfg: Dict[str, Any]) -> Dict[str, str]:
    """FastAPI's default /openapi.json, /docs, /docs/oauth2-redirect and /redoc of the
    reference app (``FastAPI(title="OpenAI API Proxy")``, oai_proxy.py:70), rendered once from
    the conformance app so the native front-end serves the same documents."""
    try:
        import json

        from fastapi.openapi.docs import get_redoc_html, get_swagger_ui_html, get_swagger_ui_oauth2_redirect_html

        from ..server.app import create_app
    except ImportError:  # fastapi absent: the routes 404, as any unknown path
        return {}
    app = create_app(lambda: cfg)
    return {
        "openapi_json": json.dumps(app.openapi(), separators=(",", ":")),
        "docs_html": get_swagger_ui_html(openapi_url=app.openapi_url, title=f"{app.title} - Swagger UI",
                                         oauth2_redirect_url=app.swagger_ui_oauth2_redirect_url,
                                         init_oauth=app.swagger_ui_init_oauth,
                                         swagger_ui_parameters=app.swagger_ui_parameters).body.decode(),
        "oauth2_redirect_html": get_swagger_ui_oauth2_redirect_html().body.decode(),
        "redoc_html": get_redoc_html(openapi_url=app.openapi_url, title=f"{app.title} - ReDoc").body.decode(),
    }


def _ca_bundle() -> str:
    """CA bundle for https upstreams: SSL_CERT_FILE, else certifi's (httpx's default), else system."""
    if os.environ.get("SSL_CERT_FILE"):
        return os.environ["SSL_CERT_FILE"]
    try:
        import certifi

        return certifi.where()
    except ImportError:
        return ""


def cluster_config(rt: RuntimeConfig, port: int, engine: str) -> Dict[str, Any]:
    """Rank / placement / exchange settings (:func:`quorum_amd.parallel.exchange.cluster_config`)."""
    from ..parallel.exchange import cluster_config as _cc

    try:
        return _cc(rt.placement, rt.exchange, rt.exchange_round_us, rt.exchange_timeout, port, engine,
                   eager_bytes=rt.exchange_eager_bytes)
    except ValueError as exc:
        raise NativeUnsupported(str(exc)) from exc


def run_native(config: str, host: str, port: int, engine: str, device: Optional[int], threads: int) -> int:
    import faulthandler

    from ..ops import native

    # a native fault is reported by the server's own handler (module+offset backtrace),
    # which then chains to this one for the Python side of the stack
    faulthandler.enable(all_threads=True)

    ext = native.require()
    cfg = load_config(config)
    d = native_config(cfg, host, port, engine, device, threads)
    return int(ext.run_server(d))
