"""GPU tests: the CDNA4 HIP stream engine vs the C++ CPU engine / python oracle.

Run on an MI355X via ``pytest -m gpu``.  Every test uses ``HipEngine`` (the fused tick
kernel): a missing extension or GPU is a hard failure here, never a silent fallback.
"""
import random

import pytest

from quorum_amd.ops import native, reference as ref
from quorum_amd.ops.engine import F_ABORTED, F_DONE, FinalizeRequest
from quorum_amd.ops.native import NativeEngine

import engine_harness as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    e = native.require()
    assert e.device_count() > 0, "no GPU visible"
    return e


def _hip(tags, **kw):
    return NativeEngine("hip", tags, device=0, **kw)


def _gpu_did_it(eng, escalations=0):
    """The HIP engine did the work itself: no stream migrated to the host path (beyond the
    `escalations` a test provokes on purpose) and every finalize ran in fused GPU items."""
    st = eng._e.kernel_stats()
    if escalations is not None:
        assert st["escalations"] == escalations, st
    assert st["fin_host"] == 0 and st["fin_items"] >= 2, st
    return st


def _check(seed, n_streams, hip_kw=None, max_piece=None, escalations=0):
    """HIP vs CPU engine on random streams; escalations=None: the case provokes host-path
    migrations (tiny tiles, content overflow), so their number is not pinned."""
    rng = random.Random(seed)
    tags = rng.sample(["think", "reason", "reasoning", "thought", "x"], rng.randint(1, 4))
    raw = [H.rand_stream(rng) for _ in range(n_streams)]
    streams = [H.split_random(rng, r, max_piece or rng.choice([3, 17, 64, 400, 5000])) for r in raw]
    filt = [rng.random() < 0.8 for _ in raw]
    emit = [rng.random() < 0.8 for _ in raw]
    tseed = rng.randint(0, 10**9)
    cpu = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(tseed))
    eng = _hip(tags, **(hip_kw or {}))
    hip = H.run_engine(eng, streams, filt, emit, random.Random(tseed))
    if escalations is not None:
        _gpu_did_it(eng, escalations)
    (c, cf, ct), (g, gf, gt) = cpu, hip
    for i, (a, b) in enumerate(zip(c, g)):
        assert a[1] == b[1], ("flags", i, raw[i])
        assert a[0] == b[0], ("sse", i, raw[i])
        assert a[2] == b[2], ("content", i, raw[i])
    assert cf == gf
    assert ct == gt


@pytest.mark.parametrize("seed", range(24))
def test_hip_matches_cpu_wide_tags(ext, seed):
    """16 tags (two MFMA column blocks), 18-33-byte tags (window prefix match + tail compare,
    near misses that differ only past the window), spaces and symbols, long holdbacks across
    tile boundaries: HIP == C++ CPU engine (== the python oracle, test_native_differential)."""
    rng = random.Random(seed)
    tags = rng.sample(H.WIDE_TAGS, rng.randint(9, 16))
    alpha = H.wide_alphabet(tags)
    raw = [H.rand_wide_stream(rng, alpha) for _ in range(rng.choice([4, 24]))]
    streams = [H.split_random(rng, r, rng.choice([3, 17, 64, 400])) for r in raw]
    filt = [rng.random() < 0.9 for _ in raw]
    emit = [rng.random() < 0.9 for _ in raw]
    tseed = rng.randint(0, 10**9)
    cpu = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(tseed))
    eng = _hip(tags)
    hip = H.run_engine(eng, streams, filt, emit, random.Random(tseed))
    assert hip == cpu, (tags, raw)
    _gpu_did_it(eng)


@pytest.mark.parametrize("seed", range(60))
def test_hip_matches_cpu_random(ext, seed):
    _check(seed, 6)


@pytest.mark.parametrize("kfast", [0, 30, 29, 27, 23, 15])
@pytest.mark.parametrize("seed", range(6))
def test_hip_fast_paths_off(ext, monkeypatch, kfast, seed):
    """Each single-wave fast path switched off in turn (QMX_KFAST: 1 S2 framing, 2 S3a, 4 S4,
    8 S6 sizing, 16 S4's VALU matcher for <= 4 candidates — off: the MFMA matcher for every
    tile): the block paths they shortcut — among them the block framing's one-scan path and
    its run-scan fallback for triple newlines (ODD_EVENTS) — give the same bytes."""
    monkeypatch.setenv("QMX_KFAST", str(kfast))
    _check(5000 + seed, 12, max_piece=5000)


@pytest.mark.parametrize("seed", range(4))
def test_hip_matches_cpu_wide_batch(ext, seed):
    """Hundreds of concurrent slots → one launch with hundreds of workgroups."""
    _check(1000 + seed, 300)


@pytest.mark.parametrize("seed", range(6))
def test_hip_clean_content_envelopes(ext, seed):
    """Printable-ASCII content without quotes or backslashes (the S6 clean path: escaped
    offsets are raw offsets, one wave per event): 1-3 digit backend indices, up to 60 events
    per tile, mixed with tiles that need escapes (the general path) in the same launch."""
    rng = random.Random(seed)
    clean = "abcdefghijklmnopqrstuvwxyz ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789.,!?-:;()<>/"
    raw, idx = [], []
    for i in range(24):
        texts = ["".join(rng.choice(clean) for _ in range(rng.randint(0, 40))) for _ in range(rng.randint(1, 60))]
        if i % 5 == 4:
            texts[rng.randrange(len(texts))] += rng.choice(['"', "\\", "\n", "\u00e9"])
        raw.append(b"".join(H.event_bytes(rng, t) for t in texts) + b"data: [DONE]\n\n")
        idx.append(rng.choice([0, 3, 9, 10, 42, 99, 100, 123, 255]))
    streams = [H.split_random(rng, r, rng.choice([64, 400, 5000])) for r in raw]
    filt = [rng.random() < 0.5 for _ in raw]
    emit = [True] * len(raw)
    tseed = rng.randint(0, 10**9)
    cpu = H.run_engine(NativeEngine("cpu", ["think"]), streams, filt, emit, random.Random(tseed), indices=idx)
    eng = _hip(["think"])
    hip = H.run_engine(eng, streams, filt, emit, random.Random(tseed), indices=idx)
    assert hip == cpu
    _gpu_did_it(eng)


def test_hip_small_tiles_and_escalation(ext):
    """Tiny tiles force MORE/requeue and oversize-event escalation to the host path."""
    for seed in range(20):
        _check(2000 + seed, 5, hip_kw={"tile_bytes": 1024}, max_piece=3000, escalations=None)


def test_hip_content_overflow_escalates(ext):
    for seed in range(10):
        _check(3000 + seed, 4, hip_kw={"content_cap": 64}, escalations=None)


def test_hip_many_lt_candidates(ext):
    """> MAX_CAND '<' in one tile → kernel escalates; result still exact."""
    body = b"".join(H.event_bytes(random.Random(i), "<" * 200 + "<think>x</think>y") for i in range(12))
    streams = [[body]]
    rng = random.Random(5)
    c = H.run_engine(NativeEngine("cpu", ["think"]), streams, [True], [True], rng)
    g = H.run_engine(_hip(["think"]), streams, [True], [True], random.Random(5))
    assert c[0] == g[0]


def test_hip_think_stream_exact(ext):
    """The canonical split-tag stream (quorum tests/test_thinking_tag_filter.py)."""
    eng = _hip(["think"])
    slot = eng.open(0, True, True)
    outs = []
    for piece in ["Hello <thi", "nk>secret</th", "ink> World"]:
        eng.feed(slot, H.event_bytes(random.Random(0), piece))
        res, _ = eng.tick(H.CREATED)
        outs.append(b"".join(r[1] for r in res if r[0] == slot))
    assert outs[0] == ref.delta_event(0, H.CREATED, "Hello ")
    assert outs[1] == b""
    assert outs[2] == ref.delta_event(0, H.CREATED, " World")
    eng.finish(slot)
    res, _ = eng.tick(H.CREATED)
    assert any(r[0] == slot and r[2] for r in res)
    assert eng.text(slot) == "Hello  World"
    eng.release(slot)


def test_hip_classify_corpus(ext):
    """Classifier fuzz through the tick kernel (wave lexer + token grammar + fallback):
    thousands of random/truncated JSON shapes, 4 events per slot, HIP == C++ CPU engine."""
    rng = random.Random(4321)
    events = []
    for _ in range(6000):
        js = H.rand_json(rng)
        if rng.random() < 0.15:
            js = js[: rng.randint(0, len(js))]
        events.append(b"data: " + js.encode() + b"\n\n")
    events += H.ODD_EVENTS + [e for e in H.ABORT_EVENTS]
    events += [b"data: {\"choices\": [{\"delta\": {\"content\": \"\xff\"}}]}\n\n",
               b"data: \xc2\xa0{} \xe2\x80\x83\n\n",
               b"data: {\"choices\": [{\"delta\": {\"content\": \"\xed\xa0\x80\"}}]}\n\n",
               b"data: {\"choices\": [{\"delta\": {\"content\": \"" + b"\\\\" * 70 + b"\\\"x\"}}]}\n\n",
               b"data: {\"choices\": [{\"delta\": {\"content\": \"" + "é".encode() * 60 + b"\"}}]}\n\n",
               b"data: {\"choices\": [{\"delta\": {\"content\": \"" + b"x" * 63 + "é".encode() + b"\"}}]}\n\n",
               b"data: " + b"[" * 300 + b"]" * 300 + b"\n\n", b"data: " + b"[1," * 1500 + b"1" + b"]" * 1500 + b"\n\n",
               b"data: {\"choices\": [{\"delta\": {\"content\": \"big\"}}], \"n\": " + b"1" * 200 + b"}\n\n"]
    streams = [[b"".join(events[i:i + 4])] for i in range(0, len(events), 4)]
    n = len(streams)
    c = H.run_engine(NativeEngine("cpu", ["think"]), streams, [True] * n, [True] * n, random.Random(9))
    g = H.run_engine(_hip(["think"], max_slots=4096), streams, [True] * n, [True] * n, random.Random(9))
    for i in range(n):
        assert c[0][i] == g[0][i], streams[i]
    assert c[1:] == g[1:]


TPL_MIDDLES = [b"hello", b"", b"a\\nb", b"q\\\"q", b"\\\\", b"\\\\\\\\", b"x\\", b"\\u00e9", b"\\u00", b"\\ud83d\\ude00",
               "\u00e9\u4e2d".encode(), b"\xff", b"\xe4\xb8", b'", "content": "override', b'"}, "x": {"y": "',
               b"tab\there", b"<think>", b"</think>", b"\\/", b"\\q", b"a" * 300, b"\\\\" * 40 + b"\\\"",
               b"\\" * 63 + b"n", b"e\xcc\x81" * 30]


def test_hip_template_path(ext):
    """Per-stream shape template: events identical outside the content string take the
    one-compare path; every anomaly in the middle must fall back to the full parse."""
    shapes = [(b'data: {"id": "c1", "choices": [{"index": 0, "delta": {"content": "', b'"}, "finish_reason": null}]}'),
              (b'data: {"choices":[{"delta":{"content":"', b'"}}]}  '),
              (b'data:  {"choices": [{"delta": {"role": "assistant", "content": "', b'", "x": 1}}]}')]
    rng = random.Random(77)
    streams = []
    for sh in range(30):
        pre, suf = shapes[sh % len(shapes)]
        evs = [pre + b"warm" + suf + b"\n\n"]
        for _ in range(40):
            evs.append(pre + rng.choice(TPL_MIDDLES) + suf + b"\n\n")
        body = b"".join(evs)
        streams.append(H.split_random(rng, body, rng.choice([50, 400, 5000])))
    n = len(streams)
    tags = ["think"]
    c = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(3))
    g = H.run_engine(_hip(tags), streams, [True] * n, [True] * n, random.Random(3))
    for i in range(n):
        assert c[0][i] == g[0][i], i
    assert c[1:] == g[1:]


FIN_PIECES = ["<think>", "</think>", "<THINK>", "</Think>", "<reason>", "</reason>", "<reasoning>", "</reasoning>",
              "<thought>", "</thought>", "<thi", "nk>", "x", " ", "\n", "\u3000", "\u00a0", "\u2003", "\u0085",
              "\u00e9", "\u4e2d", "\U0001f600", "\ud83d", "\"", "\\", "\t", "\x01", "<", ">", "/", "</"]


@pytest.mark.parametrize("seed", range(6))
def test_hip_finalize_kernel_matches_cpu(ext, seed):
    """K3 strip + K4 join + K5 encode on the GPU vs the C++ host algorithms (both
    finalize kinds), over unfiltered texts full of tags, Unicode whitespace and escapes."""
    rng = random.Random(500 + seed)
    tags = ["think", "reason", "reasoning", "thought"]
    n = rng.choice([1, 2, 3, 8, 9])
    streams = []
    for _ in range(n):
        body = b""
        for _ in range(rng.randint(0, 12)):
            txt = "".join(rng.choice(FIN_PIECES) for _ in range(rng.randint(1, 30)))
            body += H.event_bytes(rng, txt)
        streams.append([body] if body else [])
    big = "".join(rng.choice(FIN_PIECES) for _ in range(1200))  # ~5 KB text, hundreds of tokens
    streams.append([H.event_bytes(rng, big)])
    m = len(streams)
    filt = [False] * m  # keep tags in the content so the final strip has work
    for strip in (True, False):
        for joiner in ("\n---\n", "", "\u00e9|"):
            c = H.run_engine(NativeEngine("cpu", tags), streams, filt, [True] * m, random.Random(1),
                             strip_final=strip, joiner=joiner)
            eng = _hip(tags)
            g = H.run_engine(eng, streams, filt, [True] * m, random.Random(1), strip_final=strip, joiner=joiner)
            assert c[1] == g[1], (strip, joiner)
            assert c[2] == g[2], (strip, joiner)
    st = eng._e.kernel_stats()
    assert st["fin_items"] >= 1, st  # the GPU path ran (texts-kind with 9+ texts falls back)


@pytest.mark.parametrize("seed", range(3))
def test_hip_finalize_long_texts_many_texts_on_gpu(ext, seed):
    """K3 without host bail-outs: texts of ~100 KB carrying > 4096 tag tokens (unclosed opens,
    cross-type closes, nesting) and texts-kind requests with more than 8 texts all finalize
    on the GPU (fin_host stays 0) and match the C++ host algorithms byte for byte."""
    rng = random.Random(900 + seed)
    tags = ["think", "reason", "reasoning", "thought"]
    streams = []
    for k in range(12):
        n_events = 130 if k < 2 else rng.randint(1, 3)  # 130 x 200 pieces: ~100 KB of content
        evs = ["".join(rng.choice(FIN_PIECES) for _ in range(200)) for _ in range(n_events)]
        if k == 0:
            assert "".join(evs).count("<") > 4096
        streams.append([b"".join(H.event_bytes(rng, t) for t in evs[i:i + 8]) for i in range(0, n_events, 8)])
    m = len(streams)
    filt = [False] * m
    for strip in (True, False):
        c = H.run_engine(NativeEngine("cpu", tags), streams, filt, [True] * m, random.Random(1),
                         strip_final=strip, joiner="\n--\n")
        eng = _hip(tags, content_cap=1 << 18, max_slots=64)
        g = H.run_engine(eng, streams, filt, [True] * m, random.Random(1), strip_final=strip, joiner="\n--\n")
        assert c[1] == g[1], strip
        assert c[2] == g[2], strip
        st = eng._e.kernel_stats()
        assert st["fin_items"] >= 2 and st["fin_host"] == 0 and st["escalations"] == 0, st
        assert st["fin_separate_launches"] == 0, st  # finalize rides the tick launch


@pytest.mark.parametrize("seed", range(4))
def test_hip_tagdense_matches_cpu(ext, seed):
    """tools/kbench.py's tag-dense shape (120 '<' per 5 KB stream: tags, near misses, nested
    and split think blocks — eight MFMA match groups per tile) through the HIP engine, split
    at random points, byte-equal to the C++ CPU engine with no host escalation."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import kbench

    rng = random.Random(900 + seed)
    tags = ["think", "reason", "reasoning", "thought"]
    raw = kbench.tagdense_stream(tokens=rng.randint(10, 40))
    streams = [H.split_random(rng, raw, rng.choice([64, 400, 6000])) for _ in range(6)]
    n = len(streams)
    cpu = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(seed))
    eng = _hip(tags)
    hip = H.run_engine(eng, streams, [True] * n, [True] * n, random.Random(seed))
    assert hip == cpu
    _gpu_did_it(eng)


class _Poisoned:
    """An engine whose result records are refilled before every tick with the sequence number
    that tick will publish (done, nothing consumed, no output) — what pinned pages recycled
    from an earlier engine in the same process hold.  Completion must still come from this
    tick's own kernel writes."""

    def __init__(self, eng):
        self._eng = eng

    def __getattr__(self, k):
        return getattr(self._eng, k)

    def tick(self, created):
        self._eng._e.debug_poison_results(1)
        return self._eng.tick(created)


@pytest.mark.parametrize("control", [False, True])
@pytest.mark.parametrize("persistent", ["1", "0"])
def test_hip_stale_result_records(ext, monkeypatch, persistent, control):
    """Root cause of the one mislabelled delta of profiles/r4/q (backend 1's text under
    chatcmpl-parallel-0, lanes mode): sequence numbers restart with every engine, and a new
    engine's hipHostMalloc'd result records could hold a freed engine's records, so a record
    already equal to a new tick's number "completed" it at post time.  prepare() now clears
    every record the tick publishes.  control: the clearing switched off
    (QMX_DEBUG_STALE_RECORDS, the code before the fix) — the results must then differ, so
    the poison reproduces the failure on demand, in one-shot and persistent launches."""
    monkeypatch.setenv("QMX_PERSISTENT", persistent)
    if control:
        monkeypatch.setenv("QMX_DEBUG_STALE_RECORDS", "1")
    differ = 0
    for seed in (31, 32, 33):
        rng = random.Random(seed)
        tags = ["think", "reason"]
        raw = [H.rand_stream(rng) for _ in range(6)]
        streams = [H.split_random(rng, r, rng.choice([17, 64, 400])) for r in raw]
        n = len(streams)
        cpu = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(seed))
        eng = _hip(tags)
        hip = H.run_engine(_Poisoned(eng), streams, [True] * n, [True] * n, random.Random(seed))
        if control:
            differ += hip != cpu
            continue
        assert hip == cpu, seed
        _gpu_did_it(eng)
    if control:  # (every tick is poisoned; a case escapes only if all its ticks beat the host's first look)
        assert differ >= 2, differ


def test_hip_engine_stats(ext):
    eng = _hip(["think"])
    slot = eng.open(0, True, True)
    eng.feed(slot, H.event_bytes(random.Random(1), "abc"))
    eng.finish(slot)
    eng.tick(H.CREATED)
    st = eng._e.kernel_stats()
    assert st["launches"] >= 1 and st["items"] >= 1
    eng.release(slot)


def test_hip_two_lanes_concurrent(ext):
    """Two tick lanes (own HIP stream + host-mapped arenas each) driven by two threads while
    a third feeds: a stream in flight on one lane is skipped by the other until settled, so
    every stream's SSE, flags and final content equal the CPU engine's."""
    import threading
    import time

    rng = random.Random(4242)
    tags = ["think", "reason"]
    raw = [H.rand_stream(rng, abort_p=0.02) for _ in range(48)]
    streams = [H.split_random(rng, r, rng.choice([7, 40, 300])) for r in raw]
    n = len(streams)
    cpu, _, _ = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(1))
    hip = _hip(tags, lanes=2)
    slots = [hip.open(i % 7, True, True) for i in range(n)]
    out = {s: [] for s in slots}
    flags = {s: 0 for s in slots}
    lock = threading.Lock()
    fed = threading.Event()
    lanes_seen = set()

    def lane_loop(lane):
        while True:
            res, _fres, taken = hip._e.tick_unsettled(H.CREATED, lane)
            with lock:
                for slot, data, fl in res:
                    out[slot].append(data)
                    flags[slot] |= fl
                if taken:
                    lanes_seen.add(lane)
            hip._e.settle(taken)
            if not taken:
                if fed.is_set() and not hip.has_work():
                    return
                time.sleep(0.0002)

    ths = [threading.Thread(target=lane_loop, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    cur = [0] * n
    while any(c <= len(s) for c, s in zip(cur, streams)):
        for i, chunks in enumerate(streams):
            if cur[i] < len(chunks):
                hip.feed(slots[i], chunks[cur[i]])
            elif cur[i] == len(chunks):
                hip.finish(slots[i])
            cur[i] += 1
        time.sleep(0.0003)
    fed.set()
    for t in ths:
        t.join(timeout=60)
        assert not t.is_alive()
    for i, s in enumerate(slots):
        assert flags[s] & (F_DONE | F_ABORTED) == cpu[i][1], ("flags", i, raw[i])
        assert b"".join(out[s]) == cpu[i][0], ("sse", i, raw[i])
        if not flags[s] & F_ABORTED:
            assert hip.text(s) == cpu[i][2], ("content", i)
    st = hip._e.kernel_stats()
    assert st["lanes"] == 2 and st["launches"] >= 2, st
    assert lanes_seen == {0, 1}


def test_hip_completion_modes(ext, monkeypatch):
    """Tick completion by polling the kernel-published sequence numbers (default) must never
    need the event fallback; the blocking-event mode (QMX_WAIT=event) gives the same bytes."""
    _check(7001, 40)
    eng = _hip(["think"])
    slot = eng.open(0, True, True)
    for i in range(20):
        eng.feed(slot, H.event_bytes(random.Random(i), "x<think>y</think>z" * (i % 3)))
        eng.tick(H.CREATED)
    st = eng._e.kernel_stats()
    assert st["launches"] >= 10 and st["poll_fallbacks"] == 0, st
    eng.release(slot)
    monkeypatch.setenv("QMX_WAIT", "event")
    _check(7002, 40)


def _oai_event(id_, created, model, delta, finish=b"null", compact=False):
    sep = b"," if compact else b", "
    col = b":" if compact else b": "
    obj = (b"{" + b'"id"' + col + b'"' + id_ + b'"' + sep + b'"object"' + col + b'"chat.completion.chunk"' + sep +
           b'"created"' + col + created + sep + b'"model"' + col + b'"' + model + b'"' + sep + b'"choices"' + col +
           b'[{"index"' + col + b"0" + sep + b'"delta"' + col + delta + sep + b'"logprobs"' + col + b"null" + sep +
           b'"finish_reason"' + col + finish + b"}]}")
    return b"data: " + obj + b"\n\n"


# hole contents: valid and invalid string bodies / numbers, type changes
HOLE_STR = [b"abc", b"", b'q\\"x', b"\\u00e9\\ud83d\\ude00", b"\xc3\xa9 ok", b"bad\xff", b"tail\\\\", b"a\\", b"x\x01y",
            b"\\uZZZZ", b"<think>", b"</think>", b"e\\nf", b"\\/", b"\xe4\xb8\xad" * 20, b"q" * 120]
HOLE_NUM = [b"1700000000", b"0", b"-1", b"01", b"1.5e3", b"-", b"1e400", b"123456789012345678901234567890123456",
            b"2.", b"-0", b"1E+2", b"true", b"null", b'"1700000000"']


def test_hip_hole_templates(ext, monkeypatch):
    """Cross-stream hole templates: fresh streams whose ids / timestamps / models / text all
    differ match an earlier launch's role, content and finish shapes without a full parse,
    and every anomaly in a hole (invalid string body, invalid or non-number scalar, a type
    change, a different spacing) falls back to the full parse — byte-identical to the CPU
    engine either way."""
    monkeypatch.setenv("QMX_STAGE_TIMING", "1")  # per-item S3 counters (hole hits)
    rng = random.Random(11)
    tags = ["think", "reason"]
    hip, cpu = _hip(tags), NativeEngine("cpu", tags)
    got = {"hip": {}, "cpu": {}}
    for rnd in range(6):
        bodies = []
        for k in range(16):
            bad = rnd >= 2 and rng.random() < 0.5  # anomalies only after templates exist
            id_ = b"chatcmpl-" + bytes(rng.choice(b"abcdef0123456789") for _ in range(rng.randint(4, 24)))
            created = rng.choice(HOLE_NUM) if bad and rng.random() < 0.3 else str(rng.randint(1, 2 ** 31)).encode()
            model = rng.choice(HOLE_STR) if bad and rng.random() < 0.3 else rng.choice([b"m-1", b"gpt-x", b"mock"])
            compact = bad and rng.random() < 0.1
            evs = [_oai_event(id_, created, model, b'{"role": "assistant", "content": ""}', compact=compact)]
            for _ in range(rng.randint(1, 12)):
                txt = rng.choice(HOLE_STR) if bad else bytes(rng.choice(b"abc <>xyz") for _ in range(rng.randint(0, 9)))
                delta = b'{"content": "' + txt + b'"}'
                if bad and rng.random() < 0.15:
                    delta = rng.choice([b'{"content": null}', b'{"content": 5}', b'{"content": ["x"]}', b"{}"])
                evs.append(_oai_event(id_, created, model, delta, compact=compact))
            evs.append(_oai_event(id_, created, model, b"{}", finish=rng.choice([b'"stop"', b'"length"', b"null"])))
            evs.append(b"data: [DONE]\n\n")
            bodies.append(b"".join(evs))
        for name, eng in (("hip", hip), ("cpu", cpu)):
            slots = [eng.open(k % 3, True, True) for k in range(len(bodies))]
            for sl, body in zip(slots, bodies):
                eng.feed(sl, body)
                eng.finish(sl)
            acc = {sl: [b"", 0] for sl in slots}
            for _ in range(50):
                res, _ = eng.tick(H.CREATED)
                for sl, data, fl in res:
                    acc[sl][0] += data
                    acc[sl][1] |= fl
                if not eng.has_work():
                    break
            for k, sl in enumerate(slots):
                got[name][(rnd, k)] = tuple(acc[sl])
                eng.release(sl)
    assert got["hip"] == got["cpu"]
    st = hip._e.kernel_stats()
    assert st.get("s3_hole_hits", 0) > 50, st  # fresh streams' role / finish / first events


def test_hip_hole_samelen(ext, monkeypatch):
    """The same-length hole fast path (ids / timestamps of one backend keep their lengths):
    fixed-length fields, and anomalies of exactly the template's lengths — escapes, a quote,
    control bytes, DEL, UTF-8, a leading zero, a sign, a fraction, an exponent, a string where
    a number was — must come out byte-identical to the CPU engine (the fast path refuses
    every one of them and the walk / full parse decides)."""
    monkeypatch.setenv("QMX_STAGE_TIMING", "1")
    rng = random.Random(21)
    tags = ["think"]
    hip, cpu = _hip(tags), NativeEngine("cpu", tags)
    id_anom = [b"abcd\\n12345678", b"abcd\\\\12345678", b'abcd\\"12345678', b"abcd\x0112345678",
               b"abcd\x7f123456789", b"abcd\xc3\xa912345678", b"abcd1234567890"]
    num_anom = [b"0123456789", b"-123456789", b"1.23456789", b"1234567e10", b'"12345678"', b"1234567890"]
    got = {"hip": {}, "cpu": {}}
    for rnd in range(5):
        bodies = []
        for k in range(24):
            bad = rnd >= 2 and rng.random() < 0.5
            id_ = b"chatcmpl-" + (rng.choice(id_anom) if bad and rng.random() < 0.5 else
                                  bytes(rng.choice(b"abcdef0123456789") for _ in range(14)))
            created = rng.choice(num_anom) if bad and rng.random() < 0.5 else str(rng.randint(10 ** 9, 2 * 10 ** 9 - 1)).encode()
            evs = [_oai_event(id_, created, b"mock", b'{"role": "assistant", "content": ""}')]
            for _ in range(rng.randint(1, 6)):
                evs.append(_oai_event(id_, created, b"mock", b'{"content": "' + bytes(rng.choice(b"abc <>xyz")
                                                                                       for _ in range(rng.randint(0, 9))) + b'"}'))
            evs.append(_oai_event(id_, created, b"mock", b"{}", finish=b'"stop"'))
            evs.append(b"data: [DONE]\n\n")
            bodies.append(b"".join(evs))
        for name, eng in (("hip", hip), ("cpu", cpu)):
            slots = [eng.open(k % 2, True, True) for k in range(len(bodies))]
            for sl, body in zip(slots, bodies):
                eng.feed(sl, body)
                eng.finish(sl)
            acc = {sl: [b"", 0] for sl in slots}
            for _ in range(50):
                res, _ = eng.tick(H.CREATED)
                for sl, data, fl in res:
                    acc[sl][0] += data
                    acc[sl][1] |= fl
                if not eng.has_work():
                    break
            for k, sl in enumerate(slots):
                got[name][(rnd, k)] = tuple(acc[sl])
                eng.release(sl)
    assert got["hip"] == got["cpu"]
    assert hip._e.kernel_stats().get("s3_hole_hits", 0) > 50


# 12-byte events next to S3a's "data: [DONE]" word compare, and longer / shorter spellings
DONE_LIKE = [b"data: [DONE]", b"data: [DONX]", b"data: {DONE}", b"data:  [DONE", b"Data: [DONE]", b"data: [done]",
             b"data:[DONE] ", b"data: [DONE] ", b"data:[DONE]", b'data: "DONE"', b"data: [DON\xc3\x89]", b"data: 123456"]


LONG_TAGS = ["extended_reasoning_block", "a_very_long_reasoning_tag_name_for_tests"]  # 24 / 40 bytes


@pytest.mark.parametrize("seed", range(3))
def test_hip_long_tag_holdback_matches_cpu(ext, seed):
    """Streamed think filter with tags longer than 16 bytes, their openings and closings cut
    at random offsets across events and ticks: held-back tails longer than the two pattern
    words the one-wave filter keeps in registers (the tag-prefix test reads the further words),
    so the streamed deltas, flags and final content equal the CPU engine's."""
    rng = random.Random(3100 + seed)
    tags = ["think"] + LONG_TAGS
    pieces = ["<think>", "</think>", "x", " word", "<", "</", "é", "<ext", "</a_very"]
    for t in LONG_TAGS:
        pieces += [f"<{t}>", f"</{t}>", f"<{t.upper()}>", f"<{t[:20]}", f"</{t[:30]}"]
    streams = []
    for _ in range(24):
        txt = "".join(rng.choice(pieces) for _ in range(rng.randint(4, 30)))
        cuts = sorted(rng.sample(range(1, len(txt)), min(len(txt) - 1, rng.randint(1, 14))))
        body = b"".join(H.event_bytes(rng, txt[a:b]) for a, b in zip([0] + cuts, cuts + [len(txt)]))
        streams.append(H.split_random(rng, body, rng.choice([60, 500, 5000])))
    n = len(streams)
    c = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(5))
    g = H.run_engine(_hip(tags), streams, [True] * n, [True] * n, random.Random(5))
    for i in range(n):
        assert c[0][i] == g[0][i], i
    assert c[1:] == g[1:]


def test_hip_done_and_twelve_byte_events(ext, monkeypatch):
    """S3a resolves an exact ``data: [DONE]`` event itself; every other event of that length
    (and the spellings the full parse strips to [DONE]) must come out as the CPU engine has
    them, mixed with hole-template role / finish events."""
    monkeypatch.setenv("QMX_STAGE_TIMING", "1")
    rng = random.Random(31)
    hip, cpu = _hip(["think"]), NativeEngine("cpu", ["think"])
    got = {"hip": {}, "cpu": {}}
    for rnd in range(4):
        bodies = []
        for k in range(20):
            id_ = b"chatcmpl-" + bytes(rng.choice(b"abcdef0123456789") for _ in range(14))
            evs = [_oai_event(id_, b"1700000000", b"mock", b'{"role": "assistant", "content": ""}')]
            for _ in range(rng.randint(1, 5)):
                evs.append(_oai_event(id_, b"1700000000", b"mock", b'{"content": "tok"}'))
                if rnd >= 1 and rng.random() < 0.3:
                    evs.append(rng.choice(DONE_LIKE) + b"\n\n")
            evs.append(_oai_event(id_, b"1700000000", b"mock", b"{}", finish=b'"stop"'))
            evs.append((rng.choice(DONE_LIKE) if rnd >= 1 and rng.random() < 0.5 else b"data: [DONE]") + b"\n\n")
            bodies.append(b"".join(evs))
        for name, eng in (("hip", hip), ("cpu", cpu)):
            slots = [eng.open(k % 2, True, True) for k in range(len(bodies))]
            for sl, body in zip(slots, bodies):
                eng.feed(sl, body)
                eng.finish(sl)
            acc = {sl: [b"", 0] for sl in slots}
            for _ in range(50):
                res, _ = eng.tick(H.CREATED)
                for sl, data, fl in res:
                    acc[sl][0] += data
                    acc[sl][1] |= fl
                if not eng.has_work():
                    break
            for k, sl in enumerate(slots):
                got[name][(rnd, k)] = tuple(acc[sl])
                eng.release(sl)
    assert got["hip"] == got["cpu"]
    assert hip._e.kernel_stats()["escalations"] == 0
