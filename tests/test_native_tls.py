"""https upstreams in the native data plane (OpenSSL, non-blocking handshake on epoll).

Like the reference's httpx client, the peer certificate and host name are verified against
a CA bundle (certifi by default, SSL_CERT_FILE here: a throwaway self-signed CA), TLS
connections are pooled with keep-alive, and an untrusted certificate is a connection failure.
"""
import os
import shutil
import subprocess

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, completion, sse_stream
from live_upstream import LiveUpstream, native_server

pytestmark = [pytest.mark.skipif(not native.available(), reason="native extension not built"),
              pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")]
AUTH = {"Authorization": "Bearer k"}
MSG = [{"role": "user", "content": "hi"}]
BLOCK = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": True,
         "thinking_tags": ["think"], "skip_final_aggregation": False}


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    crt, key = str(d / "c.pem"), str(d / "k.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt,
                    "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost"],
                   check=True, capture_output=True)
    return crt, key


def _run(cfg, req, n=1):
    with native_server(cfg) as port:
        with httpx.Client(base_url=f"http://127.0.0.1:{port}") as c:
            return [c.post("/chat/completions", json=req, headers=AUTH, timeout=30) for _ in range(n)]


def test_https_backends_match_http(cert, monkeypatch):
    live = LiveUpstream()
    beh = {"a": ("stream", 200, sse_stream(["<think>x</think>Hel", "lo"])), "b": ("stream", 200, sse_stream(["TLS"]))}
    plain = {k: live.serve(k, v) for k, v in beh.items()}
    tls = {k: live.serve(k + "s", v, tls=cert) for k, v in beh.items()}
    try:
        req = {"messages": MSG, "stream": True}
        cfg_http = cfg_parallel(2, block=BLOCK)
        cfg_https = cfg_parallel(2, block=BLOCK)
        for i, k in enumerate(("a", "b")):
            cfg_http["primary_backends"][i]["url"] = f"http://127.0.0.1:{plain[k]}/v1"
            cfg_https["primary_backends"][i]["url"] = f"https://127.0.0.1:{tls[k]}/v1"
        monkeypatch.setenv("SSL_CERT_FILE", cert[0])
        ref = _run(cfg_http, req)[0]
        got = _run(cfg_https, req, n=12)  # keep-alive: pooled TLS sessions are reused
        for r in got:
            assert r.status_code == 200
            assert r.text.replace('"created": ', "") .split() and _final(r.text) == _final(ref.text) == "Hello\n\n--\nTLS"
        # non-streaming through TLS
        cfg_ns = cfg_parallel(2, block=BLOCK)
        for i in range(2):
            cfg_ns["primary_backends"][i]["url"] = f"https://127.0.0.1:{tls['a']}/v1"
        live.behaviours["as"] = ("json", 200, completion("<think>t</think>ok"))
        r = _run(cfg_ns, {"messages": MSG})[0]
        assert r.status_code == 200 and r.json()["choices"][0]["message"]["content"] == "ok\n--\nok"
    finally:
        live.close()


def test_https_untrusted_certificate_fails(cert, monkeypatch, tmp_path):
    live = LiveUpstream()
    p = live.serve("x", ("stream", 200, sse_stream(["secret"])), tls=cert)
    try:
        other = tmp_path / "empty.pem"  # a CA bundle that does not contain our certificate
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(tmp_path / "o.key"),
                        "-out", str(other), "-days", "1", "-subj", "/CN=other"], check=True, capture_output=True)
        monkeypatch.setenv("SSL_CERT_FILE", str(other))
        cfg = cfg_parallel(2, block=BLOCK)
        for b in cfg["primary_backends"]:
            b["url"] = f"https://127.0.0.1:{p}/v1"
        r = _run(cfg, {"messages": MSG, "stream": True})[0]
        assert r.status_code == 200
        assert "secret" not in r.text and "All backends failed" in r.text
    finally:
        live.close()


def _final(text):
    import json
    for seg in text.split("\n\n"):
        if '"chatcmpl-parallel-final"' in seg:
            return json.loads(seg[6:])["choices"][0]["delta"]["content"]
    return None
