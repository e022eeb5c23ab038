"""Loader for the native extension ``quorum_amd/_qmx*.so`` (C++ host library + CDNA4 kernels).

The extension is built in-tree by ``python -m quorum_amd.ops.build`` (or
``__graft_entry__.build()``).  On a GPU box a missing extension is an error, never a
silent fallback: :func:`require` raises with the build command.
"""
from __future__ import annotations

import importlib
import os
from typing import Callable, List, Optional, Sequence

_ext = None
_err: Optional[BaseException] = None


def _load():
    global _ext, _err
    if _ext is not None or _err is not None:
        return _ext
    try:
        _ext = importlib.import_module("quorum_amd._qmx")
    except BaseException as exc:  # noqa: BLE001
        _err = exc
    return _ext


def available() -> bool:
    return _load() is not None


def require():
    ext = _load()
    if ext is None:
        raise RuntimeError(
            "quorum_amd native extension is not built (python -m quorum_amd.ops.build): "
            f"{_err!r}")
    return ext


def gpu_available() -> bool:
    """True when the HIP runtime sees a device (does not initialise torch)."""
    if os.environ.get("QMX_FORCE_CPU") == "1":
        return False
    ext = _load()
    if ext is None:
        return False
    try:
        return ext.device_count() > 0
    except Exception:  # noqa: BLE001
        return False


def strip_fn(tags: Sequence[str]) -> Callable[[str, bool], str]:
    ext = require()
    stripper = ext.Stripper([t.lower() for t in tags])

    def _strip(text, on):
        if not on:
            return text
        if not isinstance(text, str):
            raise TypeError(f"expected string or bytes-like object, got '{type(text).__name__}'")
        return stripper.strip(text.encode("utf-8", "surrogatepass")).decode("utf-8", "surrogatepass")

    return _strip


class NativeEngine:
    """Python face of the C++ engines (``cpu`` = host library, ``hip`` = GPU tick kernels)."""

    def __init__(self, kind: str, tags: Sequence[str], device: Optional[int] = None,
                 tile_bytes: int = 16384, max_slots: int = 8192, content_cap: int = 1 << 20, lanes: int = 1,
                 grid=None, door: int = -1, ndoors: int = 1):
        ext = require()
        self.kind = kind
        self.name = kind
        self.tags: List[str] = list(tags)
        low = []
        for t in tags:
            t = t.lower()
            if t not in low:
                low.append(t)
        if kind == "hip":
            if ext.device_count() <= 0:
                raise RuntimeError("engine 'hip' requested but no GPU is visible")
            if device is None:
                device = int(os.environ.get("LOCAL_RANK", "0")) % max(ext.device_count(), 1)
            # grid: a HipGrid (loop ticks) — this engine posts its ticks into door `door` of it
            self._e = ext.HipEngine(low, device, tile_bytes, max_slots, content_cap, lanes, grid, door, ndoors)
            self.offload = True
        else:
            self._e = ext.CpuEngine(low)
            self.offload = False
        self.open = self._e.open
        self.feed = self._e.feed
        self.finish = self._e.finish
        self.release = self._e.release
        self.has_work = self._e.has_work

    def submit_finalize(self, req) -> int:
        return self._e.submit_finalize(list(req.slots), bool(req.strip), req.kind == "texts",
                                       req.joiner.encode("utf-8", "surrogatepass"), int(req.created))

    def tick(self, created: int):
        results, fres = self._e.tick(int(created))
        out = []
        for fid, kind, payload in fres:
            if kind == 0:
                out.append((fid, None))
            elif kind == 1:
                out.append((fid, payload))
            else:
                out.append((fid, [p.decode("utf-8", "surrogatepass") for p in payload]))
        return results, out

    def text(self, slot: int) -> str:
        return self._e.text(slot).decode("utf-8", "surrogatepass")

    def stats(self) -> dict:
        return dict(self._e.stats())
