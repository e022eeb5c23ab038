"""Shared differential harness: drive any stream engine with the same upstream byte streams.

Used by the CPU differential tests and the GPU (HIP engine) tests: every engine must
produce byte-identical SSE output per stream, identical DONE/ABORT flags and identical
final (filtered) content.
"""
from __future__ import annotations

import json
import random
from typing import Dict, List, Sequence, Tuple

from quorum_amd.ops.engine import F_ABORTED, F_DONE, FinalizeRequest, PyEngine

CREATED = 1700000000

TAGS_POOL = ["think", "reason", "reasoning", "thought", "Thought", "x", "ab", "t_1", "a-b"]
ALPHABET = ["<", "<", ">", "/", "think", "THINK", "reason", "reasoning", "thought", "ab", "x", " ", "\n",
            "\\", '"', "é", "😀", "a", "Z", "</", "<th", "ink>", "</think>", "<think>", "<reason>", "</reason>",
            "\t", " ", "\x01", " ", "0"]


def rand_text(rng: random.Random, n: int) -> str:
    return "".join(rng.choice(ALPHABET) for _ in range(n))


# the widest tag set the native engines take (qmx_text.h): 16 distinct tags, long ones
# (18-33 bytes: patterns past the 16-byte MFMA window, including two that share their first
# 28 bytes), spaces and ASCII symbols that are literal in quorum's regex
WIDE_TAGS = ["think", "reason", "reasoning", "thought", "internal_monologue", "scratch pad", "a=b", "x#1",
             "chain_of_thought_reasoning_v2", "chain_of_thought_reasoning_v3", "plan!", "t", "reflection",
             "self-critique:draft", "q&a", "analysis_of_the_problem_statement"]


def wide_alphabet(tags: Sequence[str]) -> List[str]:
    """Pieces that build whole, case-varied, split and near-miss tags of `tags` (a near miss
    differs in its last name byte: it passes a 16-byte window test and fails the tail)."""
    out = ["<", "</", ">", " ", "\n", "é", "😀", "a", "Z", "0", '"', "\\"]
    for t in tags:
        h = len(t) // 2
        out += [f"<{t}>", f"</{t}>", f"<{t.upper()}>", f"</{t.title()}>", "<" + t[:h], t[h:] + ">", "</" + t[:h],
                f"<{t[:-1]}~>", f"</{t[:-1]}~>", t]
    return out


def rand_wide_text(rng: random.Random, n: int, alphabet: Sequence[str]) -> str:
    return "".join(rng.choice(alphabet) for _ in range(n))


def rand_wide_stream(rng: random.Random, alphabet: Sequence[str]) -> bytes:
    parts = [event_bytes(rng, rand_wide_text(rng, rng.randint(0, 10), alphabet)) for _ in range(rng.randint(1, 12))]
    parts.append(b"data: [DONE]\n\n")
    return b"".join(parts)


def event_bytes(rng: random.Random, content) -> bytes:
    """One upstream SSE event with a random (valid) JSON shape around `content`."""
    delta = {"content": content}
    if rng.random() < 0.2:
        delta = {"role": "assistant", **delta}
    ev = {"id": "c", "object": "chat.completion.chunk", "choices": [{"index": 0, "delta": delta}]}
    if rng.random() < 0.3:
        ev["choices"][0]["finish_reason"] = None
    s = json.dumps(ev, ensure_ascii=rng.random() < 0.5)
    if rng.random() < 0.1:
        s = s.replace(", ", ",").replace(": ", ":")
    try:
        b = s.encode()
    except UnicodeEncodeError:  # lone surrogate: only the escaped form is valid UTF-8
        b = json.dumps(ev).encode()
    return b"data: " + b + b"\n\n"


ODD_EVENTS = [
    b"data: [DONE]\n\n", b": keepalive\n\n", b"event: ping\n\n", b"data: {bad}\n\n", b"data:{}\n\n",
    b"data: {\"choices\": []}\n\n", b"data: {\"choices\": [{\"delta\": {}}]}\n\n",
    b"data: {\"choices\": [{\"delta\": {\"role\": \"assistant\"}}]}\n\n",
    b"data: {\"choices\": [{\"finish_reason\": \"stop\", \"delta\": {}}]}\n\n",
    b"\n\n\n", b"data: {\"choices\": 0}\n\n", b"data: \"no choices here\"\n\n",
    b"data: [1, 2]\n\n", b"data: {\"usage\": {\"total_tokens\": 3}, \"choices\": []}\n\n",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"a\", \"content\": \"dup\"}}]}\n\n",
    b"data:  \t{\"choices\": [{\"delta\": {\"content\": \"ws\"}}]} \n\n",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"\\ud83d\\ude00\\ud800x\"}}]}\n\n",
]
ABORT_EVENTS = [
    b"data: {\"choices\": [{\"delta\": {\"content\": null}}]}\n\n",
    b"data: {\"choices\": [{\"delta\": {\"content\": 5}}]}\n\n",
    b"data: {\"choices\": {\"a\": 1}}\n\n", b"data: 7\n\n", b"data: null\n\n",
    b"data: {\"choices\": [\"x\"]}\n\n",
]


def rand_stream(rng: random.Random, abort_p: float = 0.05) -> bytes:
    parts = []
    if rng.random() < 0.2:
        parts.append(rng.choice([b" ", b"\n", b"\n\n", b"\xc2\xa0"]))
    for _ in range(rng.randint(0, 14)):
        r = rng.random()
        if r < 0.7:
            parts.append(event_bytes(rng, rand_text(rng, rng.randint(0, 12))))
        elif r < 0.7 + abort_p:
            parts.append(rng.choice(ABORT_EVENTS))
        else:
            parts.append(rng.choice(ODD_EVENTS))
    if rng.random() < 0.7:
        parts.append(b"data: [DONE]\n\n")
    elif rng.random() < 0.5:
        parts.append(event_bytes(rng, rand_text(rng, 5))[:-2])  # unterminated last event
    return b"".join(parts)


def split_random(rng: random.Random, data: bytes, max_piece: int = 40) -> List[bytes]:
    out, i = [], 0
    while i < len(data):
        k = rng.randint(1, max_piece)
        out.append(data[i:i + k])
        i += k
    return out


def run_engine(engine, streams: Sequence[List[bytes]], filt: Sequence[bool], emit: Sequence[bool],
               rng: random.Random, strip_final: bool = True, joiner: str = "\n---\n", indices=None):
    """Feed chunk lists round-robin with ticks at random points; return per-stream results.
    ``indices``: each stream's backend index (default i % 7)."""
    slots = [engine.open(indices[i] if indices else i % 7, filt[i], emit[i]) for i in range(len(streams))]
    out: Dict[int, List[bytes]] = {s: [] for s in slots}
    flags: Dict[int, int] = {s: 0 for s in slots}
    cursors = [0] * len(streams)
    fins = []

    def do_tick():
        results, fres = engine.tick(CREATED)
        for slot, data, fl in results:
            out[slot].append(data)
            flags[slot] |= fl
        fins.extend(fres)

    active = True
    while active:
        active = False
        for i, chunks in enumerate(streams):
            if cursors[i] < len(chunks):
                engine.feed(slots[i], chunks[cursors[i]])
                cursors[i] += 1
                active = True
            elif cursors[i] == len(chunks):
                engine.finish(slots[i])
                cursors[i] += 1
        if rng.random() < 0.5:
            do_tick()
    for _ in range(1000):
        if not engine.has_work():
            break
        do_tick()
    good = [s for s in slots if not (flags[s] & F_ABORTED)]
    fid = engine.submit_finalize(FinalizeRequest(good, strip_final, "event", joiner, CREATED))
    fid2 = engine.submit_finalize(FinalizeRequest(good, strip_final, "texts"))
    for _ in range(10):
        if not engine.has_work():
            break
        do_tick()
    fin = dict(fins)
    res = []
    for s in slots:
        res.append((b"".join(out[s]), flags[s] & (F_DONE | F_ABORTED),
                    engine.text(s) if not (flags[s] & F_ABORTED) else ""))
    for s in slots:
        engine.release(s)
    return res, fin.get(fid), fin.get(fid2)


def python_engine(tags):
    return PyEngine(tags)


# random JSON documents around quorum's choices[0].delta.content path (classifier fuzzing)
JSON_ATOMS = ['"choices"', '"delta"', '"content"', '"x"', '""', "0", "0.0", "-0", "1e-400", "1", "true",
              "false", "null", "NaN", "-Infinity", '"cho\\u0069ces"', '"content here"', '"\\ud800"']


def rand_json(rng, depth=0):
    r = rng.random()
    if depth == 0 and r < 0.35:
        inner = rng.choice(JSON_ATOMS + ['"hi <think>x"', '"a\\u00e9\\n"'])
        delta = rng.choice(['{"content": %s}', '{"role": "assistant", "content": %s}', '{"content": %s, "x": [1]}',
                            '%s', '{"content": {"a": %s}}']) % inner
        c0 = rng.choice(['{"delta": %s}', '{"index": 0, "delta": %s, "finish_reason": null}', '[%s]']) % delta
        return rng.choice(['{"choices": [%s]}', '{"id": "x", "choices": [%s, 1]}', '{"choices": %s}']) % c0
    if depth > 4 or r < 0.3:
        return rng.choice(JSON_ATOMS)
    if r < 0.65:
        keys = rng.sample(['"choices"', '"delta"', '"content"', '"index"', '"c\\u006fntent"', '"role"'],
                          rng.randint(0, 3))
        return "{" + ", ".join(f"{k}: {rand_json(rng, depth + 1)}" for k in keys) + "}"
    return "[" + ", ".join(rand_json(rng, depth + 1) for _ in range(rng.randint(0, 3))) + "]"
