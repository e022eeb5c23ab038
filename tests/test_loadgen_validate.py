"""qmx_loadgen's response validator: the bench only counts responses that satisfy the
proxy's event contract (reference src/quorum/oai_proxy.py:530-885).  A tiny HTTP server
returns crafted SSE bodies; each defect must be counted as invalid."""
from __future__ import annotations

import json
import subprocess
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from quorum_amd.ops import build as qbuild

TEXT = "Hello wörld \"q\" \\ 😀"


def ev(eid, delta, finish=None):
    d = {"id": eid, "object": "chat.completion.chunk", "created": 17, "model": "parallel-proxy",
         "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}
    return "data: " + json.dumps(d) + "\n\n"


def good_body(final=None):
    out = ev("chatcmpl-parallel", {"role": "assistant"})
    out += ev("chatcmpl-parallel-1", {"content": TEXT[:5]})
    out += ev("chatcmpl-parallel-0", {"content": TEXT[:7]})
    out += ev("chatcmpl-parallel-0", {"content": TEXT[7:]})
    out += ev("chatcmpl-parallel-1", {"content": TEXT[5:]})
    if final is not None:
        out += ev("chatcmpl-parallel-final", {"content": final}, "stop")
    return out + "data: [DONE]\n\n"


def _serve(body: str, status=200):
    data = body.encode()

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_POST(self):
            self.rfile.read(int(self.headers.get("content-length", "0")))
            self.send_response(status)
            self.send_header("content-type", "text/event-stream")
            self.send_header("transfer-encoding", "chunked")
            self.end_headers()
            for i in range(0, len(data), 37):  # odd chunk boundaries: split events / UTF-8
                c = data[i:i + 37]
                self.wfile.write(b"%x\r\n%s\r\n" % (len(c), c))
            self.wfile.write(b"0\r\n\r\n")
            self.wfile.flush()

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def _spec(tmp_path, final="absent", modes=("exact", "exact")):
    lines = ["role 1", "done 1"]
    for i, m in enumerate(modes):
        lines.append(f"stream chatcmpl-parallel-{i} {m} {TEXT.encode().hex()}")
    lines.append("final absent" if final == "absent" else "final any " + " ".join(x.encode().hex() for x in final))
    lines.append("error absent")
    p = tmp_path / "spec.txt"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _run(body, spec, status=200, n=6):
    lg = str([t for t in qbuild.build_tools() if t.name == "qmx_loadgen"][0])
    srv = _serve(body, status)
    try:
        out = subprocess.run([lg, "--port", str(srv.server_address[1]), "--conns", "2", "--requests", str(n),
                              "--threads", "1", "--timeout", "30", "--expect", spec],
                             capture_output=True, text=True, timeout=60)
    finally:
        srv.shutdown()
        srv.server_close()
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1]), out.stderr


def test_valid_bodies_pass(tmp_path):
    r, err = _run(good_body(), _spec(tmp_path))
    assert r["completed"] == 6 and r["validated"] == 6 and r["invalid"] == 0, err
    r, err = _run(good_body(final="x\ny"), _spec(tmp_path, final=["x\ny", "z"]))
    assert r["invalid"] == 0, err


@pytest.mark.parametrize("name,body,kw", [
    ("no_done", good_body()[:-len("data: [DONE]\n\n")], {}),
    ("no_role", good_body().split("\n\n", 1)[1], {}),
    ("wrong_text", good_body().replace("Hello w", "Hellx w"), {}),
    ("missing_event", good_body().replace(ev("chatcmpl-parallel-0", {"content": TEXT[7:]}), ""), {}),
    ("extra_final", good_body(final="x"), {}),
    ("final_differs", good_body(final="nope"), {"final": ["x"]}),
    ("unknown_id", good_body().replace("chatcmpl-parallel-1", "chatcmpl-parallel-7"), {}),
    ("after_done", good_body() + ev("chatcmpl-parallel-0", {"content": "late"}), {}),
    ("bad_json", good_body().replace('"object": ', '"object" '), {}),
    ("error_event", good_body().replace("data: [DONE]", ev("error", {"content": "Error"}, "error") + "data: [DONE]"),
     {}),
])
def test_defects_are_invalid(tmp_path, name, body, kw):
    r, err = _run(body, _spec(tmp_path, **kw))
    assert r["invalid"] == r["completed"] == 6, (name, err)
    assert "invalid response" in err


def test_prefix_mode_and_status(tmp_path):
    short = good_body().replace(ev("chatcmpl-parallel-1", {"content": TEXT[5:]}), "")
    r, err = _run(short, _spec(tmp_path, modes=("exact", "prefix")))
    assert r["invalid"] == 0, err  # a stream allowed to fail may stop early
    r, _ = _run(good_body(), _spec(tmp_path), status=500)
    assert r["invalid"] == 6 and r["non200"] == 6
