"""Pure-Python semantics oracle for the text hot path.

These are the exact observable semantics the native engines (C++ CPU engine and the
CDNA4 HIP tick kernels) must reproduce byte-for-byte; tests differential-check the
native paths against this module.

* :class:`ThinkingTagFilter` — incremental think-tag filter
  (reference ``src/quorum/oai_proxy.py:262-371``; semantics: SURVEY §2.7-A).
* :func:`strip_thinking_tags` — final strip (reference ``oai_proxy.py:120-139``; §2.7-B).
* :func:`classify_event` — per-SSE-event delta extraction with quorum's exception
  semantics (reference ``oai_proxy.py:595-673``; §2.7-C).
* :class:`PyStream` — one upstream backend stream processed *incrementally*
  (framing with carry-over, leading-whitespace strip at stream start, extraction,
  filtering, SSE encoding).  This is the engine of last resort (``engine: python``)
  and the oracle for the native stream engines.
"""
from __future__ import annotations

import json
import re
from typing import Iterable, List, Optional, Tuple

DEFAULT_TAGS = ["think", "reason", "reasoning", "thought"]


class ThinkingTagFilter:
    """Incrementally removes text inside thinking tags (nesting-aware, cross-type).

    State is ``(buffer, thinking_depth)``.  At depth 0 only *open* tags are
    recognised (a close tag is literal text) and a trailing partial open tag starting
    at the LAST ``<`` is held back; at depth > 0 the earliest open or close of any
    allowed tag moves the depth (floored at 0) and nothing is emitted.
    """

    def __init__(self, tags: Iterable[str]):
        self.allowed_tags = [t.lower() for t in tags]
        alt = "|".join(self.allowed_tags)
        self._open = re.compile(f"<({alt})>", re.IGNORECASE)
        # one search for "earliest open-or-close"; on a tie the open alternative wins,
        # which is what quorum's two separate searches + `close.start() < open.start()` do.
        self._token = re.compile(f"<({alt})>|</({alt})>", re.IGNORECASE)
        self._open_forms = [f"<{t}>" for t in self.allowed_tags]
        self.buffer = ""
        self.thinking_depth = 0

    def _holdback_start(self, buf: str, lo: int) -> int:
        i = buf.rfind("<", lo)
        if i != -1:
            cand = buf[i:].lower()
            for form in self._open_forms:
                if form.startswith(cand):
                    return i
        return len(buf)

    def feed(self, text: str) -> str:
        self.buffer += text  # TypeError on non-str, exactly as quorum (drives stream abort)
        buf, pos, out = self.buffer, 0, []
        while True:
            if self.thinking_depth == 0:
                m = self._open.search(buf, pos)
                if m is None:
                    cut = self._holdback_start(buf, pos)
                    out.append(buf[pos:cut])
                    self.buffer = buf[cut:]
                    return "".join(out)
                out.append(buf[pos:m.start()])
                pos = m.end()
                self.thinking_depth = 1
            else:
                m = self._token.search(buf, pos)
                if m is None:
                    self.buffer = buf[pos:]
                    return "".join(out)
                pos = m.end()
                if m.group(1) is not None:
                    self.thinking_depth += 1
                else:
                    self.thinking_depth = max(self.thinking_depth - 1, 0)

    def flush(self) -> str:
        if self.thinking_depth > 0:
            self.buffer = ""
            return ""
        buf = self.buffer
        cut = self._holdback_start(buf, 0)
        self.buffer = ""
        return buf[:cut]


def strip_thinking_tags(content: str, tags: List[str], hide_intermediate: bool = True) -> str:
    """Final-text strip: same-tag, leftmost, non-greedy, non-nested removal + ``str.strip()``.

    Spec (reference oai_proxy.py:134-139): ``re.sub("<(tags)>.*?</\\1>", "", I|S).strip()``.
    """
    if not hide_intermediate:
        return content
    pattern = "<(" + "|".join(tags) + ")>.*?</\\1>"
    return re.sub(pattern, "", content, flags=re.IGNORECASE | re.DOTALL).strip()


# ---------------------------------------------------------------------------
# SSE event encoding (json.dumps default separators, ensure_ascii=True)
# ---------------------------------------------------------------------------

def sse_data(obj) -> bytes:
    return b"data: " + json.dumps(obj).encode() + b"\n\n"


def chunk_event(event_id: str, created: int, delta: dict, finish_reason=None,
                model: str = "parallel-proxy") -> dict:
    return {
        "id": event_id,
        "object": "chat.completion.chunk",
        "created": created,
        "model": model,
        "choices": [{"index": 0, "delta": delta, "finish_reason": finish_reason}],
    }


DONE = b"data: [DONE]\n\n"
ALL_FAILED_TEXT = "Error: All backends failed to provide content"


def role_event(created: int, event_id: str = "chatcmpl-parallel", model: str = "parallel-proxy") -> bytes:
    return sse_data(chunk_event(event_id, created, {"role": "assistant"}, None, model))


def delta_event(index: int, created: int, text: str) -> bytes:
    return sse_data(chunk_event(f"chatcmpl-parallel-{index}", created, {"content": text}))


def final_event(created: int, text: str) -> bytes:
    return sse_data(chunk_event("chatcmpl-parallel-final", created, {"content": text}, "stop"))


def error_event(created: int) -> bytes:
    return sse_data(chunk_event("error", created, {"content": ALL_FAILED_TEXT}, "error"))


# ---------------------------------------------------------------------------
# Per-event classification (quorum's exception semantics)
# ---------------------------------------------------------------------------

SKIP, CONTENT, ABORT = 0, 1, 2


def classify_event(event: bytes) -> Tuple[int, Optional[str]]:
    """Classify one framed SSE event.

    SKIP    — not a ``data: `` event, ``[DONE]``, malformed JSON, no delta content.
    CONTENT — ``choices[0].delta.content`` is a str (possibly empty).
    ABORT   — any other exception in quorum's loop (``content: null``, wrong types…):
              quorum drops the rest of that backend's stream AND excludes it from the
              final (oai_proxy.py:667-673 skip :739-741).
    Invalid UTF-8 inside one event skips that event (quorum drops the whole chunk).
    """
    try:
        s = event.decode("utf-8")
    except UnicodeDecodeError:
        return SKIP, None
    if not s.strip() or not s.startswith("data: "):
        return SKIP, None
    data = s[6:].strip()
    if data == "[DONE]":
        return SKIP, None
    try:
        parsed = json.loads(data)
    except json.JSONDecodeError:
        return SKIP, None
    except Exception:  # RecursionError etc. escape quorum's inner handler
        return ABORT, None
    try:
        if "choices" in parsed and parsed["choices"]:
            delta = parsed["choices"][0].get("delta", {})
            if "content" in delta:
                c = delta["content"]
                if not isinstance(c, str):
                    return ABORT, None
                return CONTENT, c
        return SKIP, None
    except Exception:
        return ABORT, None


def _ws_prefix_len(b: bytes) -> Tuple[int, bool]:
    """Bytes of leading Unicode whitespace (str.isspace) in ``b``; second value is False
    when a trailing partial UTF-8 sequence prevents deciding yet."""
    i = 0
    n = len(b)
    while i < n:
        c = b[i]
        if c < 0x80:
            if chr(c).isspace():
                i += 1
                continue
            return i, True
        ln = 2 if c >= 0xC0 and c < 0xE0 else 3 if c >= 0xE0 and c < 0xF0 else 4 if c >= 0xF0 else 1
        if i + ln > n:
            return i, False
        try:
            ch = b[i:i + ln].decode("utf-8")
        except UnicodeDecodeError:
            return i, True
        if ch.isspace():
            i += ln
            continue
        return i, True
    return i, False


class PyStream:
    """One upstream backend stream, processed incrementally (oracle + python engine)."""

    def __init__(self, tags: List[str], filter_think: bool, emit: bool, index: int):
        self.filter = ThinkingTagFilter(tags) if filter_think else None
        self.emit = emit
        self.index = index
        self.buf = b""
        self.started = False
        self.aborted = False
        self.done = False
        self.content: List[str] = []

    def feed(self, data: bytes, created: int, eof: bool = False) -> bytes:
        if self.aborted or self.done:
            return b""
        self.buf += data
        out: List[bytes] = []
        if not self.started:
            k, decided = _ws_prefix_len(self.buf)
            self.buf = self.buf[k:]
            if not self.buf or (not decided and not eof):
                if eof:
                    self.done = True
                return b""
            self.started = True
        while not self.aborted:
            j = self.buf.find(b"\n\n")
            if j < 0:
                break
            ev, self.buf = self.buf[:j], self.buf[j + 2:]
            self._event(ev, created, out)
        if eof and not self.aborted:
            if self.buf:
                self._event(self.buf, created, out)
            self.buf = b""
            if not self.aborted and self.filter is not None:
                tail = self.filter.flush()  # always "" by construction; kept for parity
                if tail:
                    self.content.append(tail)
            self.done = True
        return b"".join(out)

    def _event(self, ev: bytes, created: int, out: List[bytes]) -> None:
        kind, c = classify_event(ev)
        if kind == SKIP:
            return
        if kind == ABORT:
            self.aborted = True
            self.buf = b""
            return
        safe = self.filter.feed(c) if self.filter is not None else c
        self.content.append(safe)
        if safe and self.emit:
            out.append(delta_event(self.index, created, safe))

    def text(self) -> str:
        return "".join(self.content)


def process_body_reference(body: bytes, tags: List[str], filter_think: bool, emit: bool,
                           index: int, created: int) -> Tuple[bytes, Optional[str]]:
    """quorum's own whole-body semantics (oai_proxy.py:578-741): decode the full body,
    ``strip().split("\\n\\n")``, per event extract and filter.  Returns (sse_out,
    final_text or None if the stream aborted).  Used as the oracle for PyStream."""
    filt = ThinkingTagFilter(tags) if filter_think else None
    out: List[bytes] = []
    content = ""
    try:
        text = body.decode()
    except UnicodeDecodeError:
        return b"", ""
    for event in text.strip().split("\n\n"):
        kind, c = classify_event(event.encode("utf-8", "surrogatepass"))
        if kind == SKIP:
            continue
        if kind == ABORT:
            return b"".join(out), None
        safe = filt.feed(c) if filt is not None else c
        content += safe
        if safe and emit:
            out.append(delta_event(index, created, safe))
    if filt is not None:
        content += filt.flush()
    return b"".join(out), content
