"""Stream engines: the per-rank batched processor behind every streaming session.

An engine owns *stream slots* (one per upstream backend stream).  Upstream bytes are
``feed``-ed into a slot's host staging as they arrive; ``tick`` processes ALL slots with
pending bytes in one batch (framing → JSON delta extraction → think filter → SSE encode)
and returns the client-ready SSE bytes per slot.  Finalisation requests (final strip +
join + final event / aggregator prompt) ride the same tick.

Engines (all byte-exact with :mod:`quorum_amd.ops.reference`):

* ``hip``    — CDNA4 HIP fused tick kernel + finalize kernel on the rank's GPU
               (``quorum_amd/csrc/qmx_hip.hip``), device-resident per-slot state.
* ``cpu``    — the same C++ host library running the sequential oracle algorithm
               (``quorum_amd/csrc/qmx_core.h``); used for CPU-only mode (BASELINE
               config 1) and as the escape hatch for exotic slots on the GPU path.
* ``python`` — :class:`PyEngine`, pure Python (last resort, arbitrary regex tags).

Reference counterpart: the per-backend loop of ``progress_streaming_aggregator``
(``src/quorum/oai_proxy.py:554-747``) and the final join (``:759-881``).
"""
from __future__ import annotations

import logging
import re
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import reference as ref

logger = logging.getLogger("quorum_amd.engine")

# result flags (shared with the native engines, see csrc/qmx_core.h)
F_DONE = 1       # stream fully processed (EOF seen, remainder framed)
F_ABORTED = 2    # quorum "exception" semantics: stream dropped & excluded from final
F_ESCALATED = 4  # native only: slot migrated to the host path


@dataclass
class FinalizeRequest:
    """Final combine of a session (reference oai_proxy.py:759-881 / 1191-1286).

    kind == "event":  strip each non-empty text (if ``strip``), join with ``joiner`` and
                      encode the ``chatcmpl-parallel-final`` SSE event (None when every
                      text was empty → caller emits the all-failed ``error`` event).
    kind == "texts":  return the stripped texts (host strings) — aggregate strategy.
    """

    slots: Sequence[int]
    strip: bool
    kind: str = "event"
    joiner: str = "\n"
    created: int = 0


# printable ASCII with no regex metacharacter (quorum alternates the tags unescaped into
# its patterns, oai_proxy.py:137, 271-274) and no '<', '>' or '/' (one tag's pattern could
# then start inside another's, which the token model of the native matchers excludes)
_PLAIN_TAG = re.compile(r"^[ -~]+$")
_NOT_PLAIN = set(".^$*+?{}[]\\|()<>/")


def native_tag_ok(tags: Sequence[str], max_tags: int = 16, max_len: int = 61) -> bool:
    """Tags the native/GPU matchers run exactly (qmx_text.h): literal printable ASCII, at
    most 16 distinct (lowercased) tags of at most 61 bytes — the MFMA matcher compares a
    16-byte window per '<' and the tail of longer patterns, two 16-pattern column blocks.
    Anything else runs on the python engine with real regex semantics."""
    low = {t.lower() for t in tags}
    return (0 < len(low) <= max_tags
            and all(_PLAIN_TAG.match(t) and not (set(t) & _NOT_PLAIN) and len(t) <= max_len for t in low))


class PyEngine:
    """Pure-Python engine (reference semantics, incremental)."""

    name = "python"
    offload = False

    def __init__(self, tags: Sequence[str]):
        self.tags = list(tags)
        self._slots: Dict[int, ref.PyStream] = {}
        self._pending: Dict[int, List[bytes]] = {}
        self._eof: set = set()
        self._next = 0
        self._finalize: List[Tuple[int, FinalizeRequest]] = []
        self._fid = 0
        self._lock = threading.Lock()

    # slot lifecycle -------------------------------------------------------
    def open(self, index: int, filter_think: bool, emit: bool) -> int:
        with self._lock:
            slot = self._next
            self._next += 1
            self._slots[slot] = ref.PyStream(self.tags, filter_think, emit, index)
            return slot

    def feed(self, slot: int, data: bytes) -> None:
        with self._lock:
            self._pending.setdefault(slot, []).append(bytes(data))

    def finish(self, slot: int) -> None:
        with self._lock:
            self._eof.add(slot)
            self._pending.setdefault(slot, [])

    def release(self, slot: int) -> None:
        with self._lock:
            self._slots.pop(slot, None)
            self._pending.pop(slot, None)
            self._eof.discard(slot)

    def submit_finalize(self, req: FinalizeRequest) -> int:
        with self._lock:
            self._fid += 1
            self._finalize.append((self._fid, req))
            return self._fid

    def has_work(self) -> bool:
        return bool(self._pending) or bool(self._finalize)

    # batch ----------------------------------------------------------------
    def tick(self, created: int):
        with self._lock:
            pending, self._pending = self._pending, {}
            eof, self._eof = self._eof, set()
            fin, self._finalize = self._finalize, []
        results = []
        for slot, chunks in pending.items():
            st = self._slots.get(slot)
            if st is None:
                continue
            was_done = st.done or st.aborted
            out = st.feed(b"".join(chunks), created, eof=slot in eof)
            flags = (F_DONE if st.done else 0) | (F_ABORTED if st.aborted else 0)
            if out or (flags and not was_done):
                results.append((slot, out, flags))
        fres = [(fid, self._run_finalize(req)) for fid, req in fin]
        return results, fres

    def text(self, slot: int) -> str:
        st = self._slots.get(slot)
        return st.text() if st is not None and not st.aborted else ""

    def _run_finalize(self, req: FinalizeRequest):
        texts = [self.text(s) for s in req.slots]
        stripped = [ref.strip_thinking_tags(t, self.tags, hide_intermediate=req.strip)
                    for t in texts if t]
        if req.kind == "texts":
            return stripped
        if not stripped:
            return None
        return ref.final_event(req.created, req.joiner.join(stripped))

    def stats(self) -> dict:
        return {"engine": self.name, "slots": len(self._slots)}


_NATIVE_CACHE: Dict[Tuple[str, Tuple[str, ...], int], object] = {}


def _py_engine(tags: Sequence[str]) -> PyEngine:
    key = ("python", tuple(tags), -1)
    eng = _NATIVE_CACHE.get(key)
    if eng is None:
        eng = PyEngine(tags)
        _NATIVE_CACHE[key] = eng
    return eng


def make_engine(kind: str, tags: Sequence[str], device: Optional[int] = None, **opts):
    """Build (and cache per process) an engine for a tag set.

    ``kind``: "auto" | "hip" | "cpu" | "python".  "hip" raises loudly when the HIP
    extension or a GPU is missing (no silent fallback on a GPU box).
    """
    tags = list(tags)
    if kind == "python" or not native_tag_ok(tags):
        if kind in ("hip", "cpu") and not native_tag_ok(tags):
            logger.warning("thinking_tags %r need regex semantics: using the python engine", tags)
        return _py_engine(tags)
    from . import native  # noqa: WPS433 - heavy import deferred

    if kind == "auto":
        if not native.available():
            logger.warning("native extension not built: using the python engine")
            return _py_engine(tags)
        kind = "hip" if native.gpu_available() else "cpu"
    key = (kind, tuple(t.lower() for t in tags), -1 if device is None else device)
    eng = _NATIVE_CACHE.get(key)
    if eng is None:
        eng = native.NativeEngine(kind, tags, device=device, **opts)
        _NATIVE_CACHE[key] = eng
    return eng

