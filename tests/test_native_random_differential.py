"""Randomised differential conformance: the native C++ data plane vs the FastAPI app.

Each seed builds a random session: 1-4 backends, concatenate or aggregate (sometimes with
an aggregator among the sources), random strategy flags, streaming or not, and per-backend
behaviours drawn from streamed bodies (random think-tag soup, escapes, non-BMP text, random
chunking, null-content aborts, malformed events), JSON completions, HTTP errors and refused
connections.  Client-visible output (per-backend SSE streams + tail, or JSON bodies) and
what each upstream received must match exactly — the same comparison as
test_native_server.py, over shapes nobody wrote by hand.
"""
import os
import random

import pytest

from quorum_amd.ops import native

import test_native_server as T
from conftest import cfg_parallel, completion, sse_chunk

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

PIECES = ["<think>", "</think>", "<reason>", "</reason>", "<THINK>", "<thi", "nk>", "</th", "hello ", "world",
          " ", "\n", "é", "😀", "\"q\"", "\\", "<", ">", "a<b", "x", "\t", "</reasoning>", "<thought>"]


def _text(rng, n):
    return "".join(rng.choice(PIECES) for _ in range(n))


def _stream_body(rng):
    chunks = []
    if rng.random() < 0.7:
        chunks.append(sse_chunk({"role": "assistant", "content": ""}))
    for _ in range(rng.randint(0, 8)):
        r = rng.random()
        if r < 0.05:
            chunks.append(sse_chunk({"content": None}))
        elif r < 0.1:
            chunks.append(b"data: {oops}\n\n")
        else:
            chunks.append(sse_chunk({"content": _text(rng, rng.randint(0, 5))}))
    chunks.append(sse_chunk({}, finish="stop"))
    if rng.random() < 0.8:
        chunks.append(b"data: [DONE]\n\n")
    raw = b"".join(chunks)
    cut = sorted(rng.sample(range(1, max(2, len(raw))), min(rng.randint(0, 6), max(0, len(raw) - 1))))
    return [raw[a:b] for a, b in zip([0] + cut, cut + [len(raw)]) if raw[a:b]]


def _behaviour(rng, stream):
    r = rng.random()
    if r < 0.08:
        return ("refuse",)
    if r < 0.16:
        return ("json", rng.choice([500, 503, 429]), {"error": {"message": _text(rng, 2)}})
    if stream:
        return ("stream", 200, _stream_body(rng))
    return ("json", 200, completion(_text(rng, rng.randint(0, 6)), cid=f"c{rng.randint(0, 9)}"))


def _scenario(seed):
    rng = random.Random(seed)
    n = rng.randint(1, 4)
    stream = rng.random() < 0.8
    strategy = "aggregate" if rng.random() < 0.3 else "concatenate"
    block = {"separator": rng.choice(["\n---\n", "\n", " | "]), "hide_intermediate_think": rng.random() < 0.7,
             "hide_final_think": rng.random() < 0.5, "thinking_tags": ["think", "reason", "reasoning", "thought"],
             "skip_final_aggregation": rng.random() < 0.3}
    if strategy == "aggregate":
        block.update({"aggregator_backend": f"LLM{rng.randint(1, n + 1)}", "include_source_names": rng.random() < 0.5,
                      "intermediate_separator": "\n\n--\n\n", "prompt_template": "P:\n{responses}\n.",
                      "include_original_query": rng.random() < 0.5})
    cfg = cfg_parallel(n, strategy=strategy, block=block)
    ups = {}
    for i in range(n):
        beh = _behaviour(rng, stream)
        if strategy == "aggregate" and block["aggregator_backend"] == f"LLM{i + 1}" and beh[0] != "refuse":
            final = _text(rng, 3)
            beh = (lambda b, f: (lambda body: b if body.get("stream") else ("json", 200, completion(f))))(beh, final)
        ups[f"b{i + 1}.test"] = beh
    req = {"messages": [{"role": "user", "content": "Q?"}], "stream": stream}
    if rng.random() < 0.15:
        req["suppress_individual_responses"] = True
    return cfg, ups, req, {"Authorization": "Bearer k"}


def run_random_session(seed, tick_mode):
    cfg, ups, req, hdrs = _scenario(seed)
    T.SCENARIOS[f"_random_{seed}"] = (cfg, ups, req, hdrs)
    try:
        T.test_native_matches_python(f"_random_{seed}", tick_mode)
    finally:
        del T.SCENARIOS[f"_random_{seed}"]


@pytest.mark.parametrize("seed", range(int(os.environ.get("QMX_RANDOM_SEEDS", "40"))))
def test_random_session_native_matches_python(seed):
    # odd seeds through the io loops' asynchronous tick path (tick_mode "loops")
    run_random_session(seed, "loops" if seed % 2 else None)
