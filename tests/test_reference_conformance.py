"""Conformance against the reference ITSELF: the unmodified quorum proxy
(/root/reference/src/quorum/oai_proxy.py, a scratch copy with only config.yaml written, as
``bench.py --impl reference`` runs it) and the native C++ server answer the same requests
against the same real-socket fake backends (tests/live_upstream.py), scenario by scenario
(the table of tests/test_native_server.py: error model, non-stream combine with the usage
sum, aggregate and its fallback, null abort, malformed events, single-backend passthrough).

The native side is otherwise pinned to the builder's FastAPI app (test_native_server.py);
this file pins it to the reference's own code.  Allowed deviations — each one a SURVEY row —
are normalised, and every normalisation is listed here:

* ``created``: the reference writes event-loop seconds (SURVEY §2.6 "created" note); both
  sides' values are set to 0.
* Event interleaving across backends: the reference emits each backend's buffered stream
  contiguously, in poll order (first bullet); qmx is incremental (§2.8, the
  allowed "truly incremental streaming" improvement).  Streaming bodies are compared per
  backend id (each backend's own event sequence, in order) plus the non-backend events in
  order (role first, final / error, [DONE] last).
* Response headers are not compared (the reference copies upstream headers onto
  passthrough responses, SURVEY §2.6 "Headers"); status and content type are.
* ``EXCEPTIONS`` below: single-backend streaming under the reference's whole-body buffering
  (its "first chunk" is the entire body: the upstream role event is kept and [DONE] comes
  twice); qmx follows the per-chunk rule the reference's own test pins.

Everything else must be equal: status, JSON bodies (errors, non-stream combines, the
passthrough's ``backend`` key), every backend's event sequence and the final / error events.
"""
from __future__ import annotations

import copy
import importlib.util
import itertools
import json
import logging
import os
import shutil
import sys

import pytest

import test_native_server as T
from live_upstream import LiveUpstream

REF_SRC = "/root/reference/src/quorum"
pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF_SRC, "oai_proxy.py")),
                                reason="reference checkout not present")

_n = itertools.count()


def _load_reference(root, cfg):
    """Import a scratch copy of the reference under a unique module name; it reads
    <root>/config.yaml (oai_proxy.py:46: three directories above the module)."""
    import yaml

    pkg = os.path.join(root, "src", "quorum")
    shutil.copytree(REF_SRC, pkg)
    with open(os.path.join(REF_SRC, "oai_proxy.py"), "rb") as a, open(os.path.join(pkg, "oai_proxy.py"), "rb") as b:
        assert a.read() == b.read()  # the reference's code, unmodified
    with open(os.path.join(root, "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    name = f"quorum_reference_{next(_n)}"
    spec = importlib.util.spec_from_file_location(name, os.path.join(pkg, "oai_proxy.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    logging.getLogger(name).setLevel(logging.WARNING)  # it logs every request body at INFO
    return name, mod


def _unload(name, root):
    sys.modules.pop(name, None)
    agg = logging.getLogger("aggregation")  # the reference adds a file handler per import
    for h in list(agg.handlers):
        if getattr(h, "baseFilename", "").startswith(str(root)):
            agg.removeHandler(h)
            h.close()


def _reference_side(cfg, ups, req, hdrs, tmp_path):
    from fastapi.testclient import TestClient

    live = LiveUpstream()
    cfg = copy.deepcopy(cfg)
    root = tmp_path / f"ref{next(_n)}"
    name = None
    try:
        for b in cfg["primary_backends"]:
            host = b["url"].split("//")[1].split("/")[0] if b["url"] else None
            if host and host in ups:
                b["url"] = f"http://127.0.0.1:{live.serve(host, ups[host])}/v1"
        name, mod = _load_reference(str(root), cfg)
        with TestClient(mod.app) as c:
            r = c.post("/chat/completions", json=req, headers=hdrs)
        return T._normalize(r.status_code, r.headers.get("content-type"), r.content), live.calls
    finally:
        live.close()
        if name:
            _unload(name, root)


def _whole_body_first_chunk(evs):
    """single-backend streaming, reference under real sockets: call_backend buffers the whole
    upstream body, so stream_with_role's "first chunk" (oai_proxy.py:911-936) is the ENTIRE
    body — json.loads fails on it ("Extra data"), the upstream's bare role event is forwarded
    instead of dropped, and saw_done stays false, so a second [DONE] is appended (:953-956).
    qmx streams incrementally (SURVEY §2.8 "Full support for streaming": the allowed fix), so
    its first chunk is the first upstream event, which is dropped when it is a bare role event
    — the behaviour the reference's own test pins with per-event chunks
    (reference tests/test_streaming.py:11-67: role, content, stop, [DONE]).  Returns the
    reference's events with exactly those two buffering artefacts removed."""
    out = list(evs)
    if len(out) > 1 and isinstance(out[1], dict):
        d = out[1]["choices"][0]["delta"]
        if d.get("role") and d.get("content", "") == "":
            del out[1]
    if out[-2:] == ["[DONE]", "[DONE]"]:
        out.pop()
    return out


# scenario -> (transform of the reference's normalised events): the documented
# exceptions.  A transform must change the reference's output (it is asserted), so an entry
# never hides an equality it does not need.
EXCEPTIONS = {
    "single_stream": ("SURVEY §2.8 'Full support for streaming' / §2.1 C10", _whole_body_first_chunk),
}


def _per_backend(evs):
    """Each backend's own event sequence + everything else in order (role, final, error, DONE)."""
    d, rest = {}, []
    for e in evs:
        eid = str(e.get("id", "")) if isinstance(e, dict) else ""
        if eid.startswith("chatcmpl-parallel-") and eid[-1].isdigit():
            d.setdefault(eid, []).append(e)
        else:
            rest.append(e)
    return d, rest


@pytest.mark.parametrize("name", sorted(T.SCENARIOS))
def test_native_matches_reference(name, tmp_path, monkeypatch):
    monkeypatch.delenv("OPENAI_API_KEY", raising=False)  # no_auth: 401 only without the env key
    cfg, ups, req, hdrs = T.SCENARIOS[name]
    ref, ref_calls = _reference_side(cfg, ups, req, hdrs, tmp_path)
    nat, nat_calls = T._native_side(cfg, ups, req, hdrs)
    assert (ref[0], ref[1]) == (nat[0], nat[1]), (name, ref, nat)
    if name in EXCEPTIONS:
        row, fix = EXCEPTIONS[name]
        fixed = fix(ref[2])
        assert fixed != ref[2], (name, row, "exception no longer needed")
        ref = (ref[0], ref[1], fixed)
    if ref[1] == "text/event-stream" and ref[0] == 200:
        assert _per_backend(ref[2]) == _per_backend(nat[2]), name
    else:
        assert ref[2] == nat[2], name
    # what the backends received: bodies (model override, suppress flag forwarded) and auth
    def calls(cs):
        return sorted((json.dumps(c["body"], sort_keys=True) if c["body"] else "", c["headers"].get("authorization") or "")
                      for c in cs)
    assert calls(ref_calls) == calls(nat_calls), name
