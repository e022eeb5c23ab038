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


def _serve(body: str, status=200, ctype="text/event-stream"):
    data = body.encode()

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_POST(self):
            self.rfile.read(int(self.headers.get("content-length", "0")))
            self.send_response(status)
            self.send_header("content-type", ctype)
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


def _run(body, spec, status=200, n=6, stream=True):
    lg = str([t for t in qbuild.build_tools() if t.name == "qmx_loadgen"][0])
    srv = _serve(body, status, "text/event-stream" if stream else "application/json")
    try:
        out = subprocess.run([lg, "--port", str(srv.server_address[1]), "--conns", "2", "--requests", str(n),
                              "--threads", "1", "--timeout", "30", "--expect", spec, "--stream", str(int(stream))],
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


MSG_TEXT = "<think>t</think>Answer é \"q\""


def completion(content=MSG_TEXT, usage=(9, 20, 29), backend="LLM1", extra=None):
    d = {"id": "c1", "object": "chat.completion", "created": 1, "model": "m",
         "choices": [{"index": 0, "message": {"role": "assistant", "content": content}, "logprobs": None,
                      "finish_reason": "stop"}]}
    if usage is not None:
        d["usage"] = {"prompt_tokens": usage[0], "completion_tokens": usage[1], "total_tokens": usage[2]}
    if backend is not None:
        d["backend"] = backend
    d.update(extra or {})
    return json.dumps(d)


def _json_spec(tmp_path):
    p = tmp_path / "spec_json.txt"
    p.write_text(f"json 1\nmessage {MSG_TEXT.encode().hex()}\nusage 9 20 29\nfield backend {b'LLM1'.hex()}\n")
    return str(p)


def test_nonstream_json_bodies(tmp_path):
    """BASELINE config 1 (non-streaming passthrough): the load generator checks the JSON
    completion — message content, usage totals and the passthrough's "backend" key."""
    r, err = _run(completion(), _json_spec(tmp_path), stream=False)
    assert r["completed"] == r["validated"] == 6 and r["invalid"] == 0, err
    for bad in (completion(content="other"), completion(usage=(9, 20, 30)), completion(usage=None),
                completion(backend="LLM2"), completion(backend=None), completion()[:-1],
                completion().replace('"choices": [{', '"choices": [{"x": 1}, {'), "[]"):
        r, err = _run(bad, _json_spec(tmp_path), stream=False)
        assert r["invalid"] == r["completed"] == 6, (bad, err)


def test_direct_mode_skips_backend_role_and_stop(tmp_path):
    """The harness-ceiling check validates a backend's own stream: role / stop events without
    content are skipped, every content byte (think block included) must arrive."""
    raw = "<think>x</think>Hi"

    def mev(delta, finish=None):
        d = {"id": "chatcmpl-mock", "object": "chat.completion.chunk", "created": 1, "model": "mock",
             "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}
        return "data: " + json.dumps(d) + "\n\n"

    body = mev({"role": "assistant", "content": ""}) + mev({"content": raw[:9]}) + mev({"content": raw[9:]})
    body += mev({}, "stop") + "data: [DONE]\n\n"
    p = tmp_path / "spec_direct.txt"
    p.write_text(f"role 0\ndone 1\nempty allowed\nstream chatcmpl-mock exact {raw.encode().hex()}\nfinal absent\n")
    r, err = _run(body, str(p))
    assert r["invalid"] == 0 and r["validated"] == 6, err
    r, err = _run(body.replace("Hi", "Ho"), str(p))
    assert r["invalid"] == 6, err
