"""Differential tests: native C++ engine vs the python oracle (SURVEY §4 implication 2).

Random upstream byte streams (random JSON shapes, escapes, split UTF-8, think tags split
at arbitrary points, quorum's exception cases) are fed to both engines with random tick
boundaries; SSE output, flags and final texts must be byte-identical.
"""
import json
import random

import pytest
from hypothesis import given, settings, strategies as st

from quorum_amd.ops import native, reference as ref
from quorum_amd.ops.native import NativeEngine

import engine_harness as H

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")


def _ext():
    return native.require()


# ---------------------------------------------------------------- event classifier
def test_classify_random_shapes():
    ext = _ext()
    rng = random.Random(1234)
    for _ in range(4000):
        js = H.rand_json(rng)
        if rng.random() < 0.1:
            js = js[: rng.randint(0, len(js))]  # truncated / malformed
        ev = b"data: " + js.encode()
        exp_kind, exp_c = ref.classify_event(ev)
        kind, c = ext.classify(ev)
        assert kind == exp_kind, (js, kind, exp_kind)
        if kind == ref.CONTENT:
            assert c.decode("utf-8", "surrogatepass") == exp_c, js


@pytest.mark.parametrize("ev", H.ODD_EVENTS + H.ABORT_EVENTS + [
    b"data: {\"choices\": [{\"delta\": {\"content\": \"a\\u0000b\\tc\"}}]}",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"raw\ttab\"}}]}",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"x\"}}]} trailing",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"x\",}}]}",
    b"data: {\"choices\": [1], \"choices\": [{\"delta\": {\"content\": \"last wins\"}}]}",
    b"data: {\"choices\": [{\"delta\": \"has content inside\"}]}",
    b"data: {\"choices\": [{\"delta\": [\"content\"]}]}",
    b"data: {\"choices\": [{\"delta\": [\"nope\"]}]}",
    b"data: [\"choices\"]",
    b"data: \"choices\"",
    b"data: {\"choices\": 1e-400}",
    b"data: {\"choices\": 0.0001}",
    b"data: {\"choices\": \"\"}",
    b"data: {\"choices\": \"s\"}",
    b"data: {\"choices\": [{\"delta\": null}]}",
    b"data: {\"choices\": [{\"delta\": {\"content\": \"\\uD83D\\uDE00\"}}]}",
    b"data: \xff\xfe",
    b"data: \xc2\xa0{\"choices\": [{\"delta\": {\"content\": \"nbsp\"}}]}\xe2\x80\x83",
    b"data: " + b"[" * 300 + b"]" * 300,
])
def test_classify_edge_cases(ev):
    kind, c = _ext().classify(ev)
    exp_kind, exp_c = ref.classify_event(ev)
    if ev.startswith(b"data: [[[["):
        exp_kind = ref.ABORT  # nesting > 256 emulates RecursionError (documented deviation)
    assert kind == exp_kind
    if kind == ref.CONTENT:
        assert c.decode("utf-8", "surrogatepass") == exp_c


# ---------------------------------------------------------------- streaming filter
@settings(max_examples=300, deadline=None)
@given(st.lists(st.sampled_from(H.ALPHABET), max_size=40), st.integers(0, 2**32 - 1),
       st.lists(st.sampled_from(H.TAGS_POOL), min_size=1, max_size=4))
def test_filter_random_chunks(pieces, seed, tags):
    text = "".join(pieces)
    rng = random.Random(seed)
    py = ref.ThinkingTagFilter(tags)
    nat = _ext().StreamFilter([t.lower() for t in tags])
    i = 0
    while i <= len(text):
        k = rng.randint(0, 6)
        chunk = text[i:i + k]
        assert nat.feed(chunk.encode()).decode() == py.feed(chunk), (text, i, k)
        i += max(k, 1)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.sampled_from(H.ALPHABET), max_size=50),
       st.lists(st.sampled_from(H.TAGS_POOL), min_size=1, max_size=4))
def test_strip_random(pieces, tags):
    text = "".join(pieces)
    exp = ref.strip_thinking_tags(text, tags)
    got = native.strip_fn(tags)(text, True)
    assert got == exp, text


# ---------------------------------------------------------------- wide tag sets
WIDE_ALPHA = H.wide_alphabet(H.WIDE_TAGS)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.sampled_from(WIDE_ALPHA), max_size=40), st.integers(0, 2**32 - 1),
       st.integers(1, len(H.WIDE_TAGS)))
def test_filter_wide_tags_random_chunks(pieces, seed, ntags):
    """16 tags, 18-33-byte tags, spaces and symbols: the native streaming filter equals the
    oracle at every chunk boundary (and the holdback of a partial long tag is exact)."""
    rng = random.Random(seed)
    tags = rng.sample(H.WIDE_TAGS, ntags)
    text = "".join(pieces)
    py = ref.ThinkingTagFilter(tags)
    nat = _ext().StreamFilter([t.lower() for t in tags])
    i = 0
    while i <= len(text):
        k = rng.randint(0, 9)
        chunk = text[i:i + k]
        assert nat.feed(chunk.encode()).decode() == py.feed(chunk), (tags, text, i, k)
        i += max(k, 1)
    assert nat.flush().decode() == py.flush()


@settings(max_examples=300, deadline=None)
@given(st.lists(st.sampled_from(WIDE_ALPHA), max_size=50), st.integers(0, 2**32 - 1))
def test_strip_wide_tags(pieces, seed):
    tags = random.Random(seed).sample(H.WIDE_TAGS, random.Random(seed).randint(1, 16))
    text = "".join(pieces)
    assert native.strip_fn(tags)(text, True) == ref.strip_thinking_tags(text, tags), (tags, text)


@pytest.mark.parametrize("seed", range(40))
def test_cpu_engine_matches_python_wide_tags(seed):
    rng = random.Random(seed)
    tags = rng.sample(H.WIDE_TAGS, rng.randint(8, 16))
    alpha = H.wide_alphabet(tags)
    raw = [H.rand_wide_stream(rng, alpha) for _ in range(4)]
    streams = [H.split_random(rng, r, rng.choice([3, 17, 64, 400])) for r in raw]
    filt, emit = [True] * 4, [True] * 4
    ts = rng.randint(0, 10**9)
    py = H.run_engine(H.python_engine(tags), streams, filt, emit, random.Random(ts))
    nat = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(ts))
    assert py == nat, (tags, raw)


def test_native_tag_rules():
    """What the native engines take (16 literal tags <= 61 bytes) and what stays on the
    python engine: regex metacharacters (quorum alternates tags unescaped), '<', '>', '/',
    non-ASCII, more than 16 distinct tags, longer tags."""
    from quorum_amd.ops.engine import native_tag_ok

    assert native_tag_ok(H.WIDE_TAGS)
    assert native_tag_ok(["x" * 61]) and not native_tag_ok(["x" * 62])
    assert native_tag_ok(H.WIDE_TAGS + ["THINK"])  # 16 distinct after lowercasing
    assert not native_tag_ok(H.WIDE_TAGS + ["extra"])
    for bad in ["a.b", "a|b", "th(ink)", "x*", "a+", "q?", "[x]", "{2}", "^a", "a$", "a\\d", "<a", "a>", "a/b",
                "é", ""]:
        assert not native_tag_ok(["think", bad]), bad
    ext = _ext()
    for bad in ["a.b", "a/b", "é"]:
        with pytest.raises(ValueError, match="regex semantics"):
            ext.StreamFilter(["think", bad])


# ---------------------------------------------------------------- whole engine
def _compare(seed, n_streams=4):
    rng = random.Random(seed)
    tags = rng.sample(["think", "reason", "reasoning", "thought", "x"], rng.randint(1, 4))
    raw = [H.rand_stream(rng) for _ in range(n_streams)]
    streams = [H.split_random(rng, r, rng.choice([3, 17, 64, 400])) for r in raw]
    filt = [rng.random() < 0.8 for _ in raw]
    emit = [rng.random() < 0.8 for _ in raw]
    tick_seed = rng.randint(0, 10**9)
    py_res = H.run_engine(H.python_engine(tags), streams, filt, emit, random.Random(tick_seed))
    nat_res = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(tick_seed))
    return raw, py_res, nat_res


@pytest.mark.parametrize("seed", range(150))
def test_cpu_engine_matches_python(seed):
    raw, (py, pyf, pyt), (nat, natf, natt) = _compare(seed)
    for i, (a, b) in enumerate(zip(py, nat)):
        assert a[1] == b[1], (i, raw[i])
        assert a[0] == b[0], (i, raw[i])
        assert a[2] == b[2], (i, raw[i])
    assert pyf == natf
    assert pyt == natt


def test_process_body_reference_agrees_with_pystream():
    """PyStream (incremental) == quorum's whole-body loop for well-formed streams."""
    rng = random.Random(99)
    for _ in range(300):
        tags = ["think", "reason"]
        body = b"".join(H.event_bytes(rng, H.rand_text(rng, rng.randint(0, 10))) for _ in range(rng.randint(1, 8)))
        st_ = ref.PyStream(tags, True, True, 0)
        out = b"".join(st_.feed(c, H.CREATED) for c in H.split_random(rng, body, 9))
        out += st_.feed(b"", H.CREATED, eof=True)
        exp_out, exp_text = ref.process_body_reference(body, tags, True, True, 0, H.CREATED)
        assert out == exp_out
        assert st_.text() == exp_text
