"""Tick scheduler: bridges the asyncio I/O world and the batched stream engine.

Upstream readers ``feed`` bytes into engine slots as they arrive.  A single ticker task
per event loop runs ``engine.tick()`` whenever work is pending: while a tick is in flight
(for the HIP engine: on a worker thread, GIL released, kernels on the rank's GPU), new
bytes accumulate for the next tick — natural adaptive batching with I/O ∥ kernel
overlap.  Outputs are dispatched to the owning session's queue.

Replaces the reference's 100 ms polling loop (``src/quorum/oai_proxy.py:554-747``).
"""
from __future__ import annotations

import asyncio
import logging
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional

from ..ops.engine import F_ABORTED, F_DONE, FinalizeRequest
from ..utils import metrics

_log = logging.getLogger("qmx.ticker")


class SessionStreams:
    """The engine slots of one client session + its output queue."""

    def __init__(self, ticker: "Ticker", n: int):
        self.ticker = ticker
        self.queue: asyncio.Queue = asyncio.Queue()
        self.slots: List[int] = []
        self.finished: Dict[int, int] = {}  # slot -> flags
        self.failed: set = set()
        self.n = n

    def all_finished(self) -> bool:
        return len(self.finished) + len(self.failed) >= self.n

    def on_output(self, slot: int, data: bytes, flags: int) -> None:
        if data:
            self.queue.put_nowait(data)
        if flags & (F_DONE | F_ABORTED):
            self.finished[slot] = flags
            if self.all_finished():
                self.queue.put_nowait(None)

    def fail(self, slot: int) -> None:
        if slot in self.finished or slot in self.failed:
            return
        self.failed.add(slot)
        if self.all_finished():
            self.queue.put_nowait(None)

    def good_slots(self) -> List[int]:
        """Slots contributing to the final (config order); failed/aborted excluded."""
        return [s for s in self.slots
                if s not in self.failed and not (self.finished.get(s, 0) & F_ABORTED)]


class Ticker:
    def __init__(self, engine, loop: asyncio.AbstractEventLoop):
        self.engine = engine
        self.loop = loop
        self._owners: Dict[int, SessionStreams] = {}
        self._futures: Dict[int, asyncio.Future] = {}
        self._wake = asyncio.Event()
        self._pool: Optional[ThreadPoolExecutor] = (
            ThreadPoolExecutor(max_workers=1, thread_name_prefix="qmx-tick") if engine.offload else None)
        self._task = loop.create_task(self._run())
        self.ticks = 0
        self.failures = 0  # engine ticks that raised (the ticker survives them)

    # session API ------------------------------------------------------------
    def open_session(self, n: int, filter_think: bool, emit: bool) -> SessionStreams:
        sess = SessionStreams(self, n)
        for i in range(n):
            slot = self.engine.open(i, filter_think, emit)
            sess.slots.append(slot)
            self._owners[slot] = sess
        return sess

    def feed(self, slot: int, data: bytes) -> None:
        self.engine.feed(slot, data)
        self._wake.set()

    def finish(self, slot: int) -> None:
        self.engine.finish(slot)
        self._wake.set()

    def release(self, sess: SessionStreams) -> None:
        for s in sess.slots:
            self._owners.pop(s, None)
            self.engine.release(s)

    async def finalize(self, req: FinalizeRequest):
        fid = self.engine.submit_finalize(req)
        fut = self.loop.create_future()
        self._futures[fid] = fut
        self._wake.set()
        return await fut

    # loop -----------------------------------------------------------------
    async def _run(self) -> None:
        while True:
            await self._wake.wait()
            self._wake.clear()
            if not self.engine.has_work():
                continue
            created = int(time.time())
            t0 = time.perf_counter()
            try:
                if self._pool is not None:
                    results, fres = await self.loop.run_in_executor(self._pool, self.engine.tick, created)
                else:
                    results, fres = self.engine.tick(created)
            except Exception as exc:  # noqa: BLE001 - never kill the ticker; fail the waiters
                self.failures += 1
                _log.error("engine tick failed (%s); failing the sessions in flight", exc)
                for fut in self._futures.values():
                    if not fut.done():
                        fut.set_exception(exc)
                self._futures.clear()
                # the batch's outputs are lost: end every live stream (as failed) so no
                # session waits for results that will never come; new sessions keep working
                for slot, owner in list(self._owners.items()):
                    owner.fail(slot)
                continue  # the next feed wakes the ticker again (no busy retry of a failing tick)
            self.ticks += 1
            metrics.observe_tick(time.perf_counter() - t0, len(results))
            for slot, data, flags in results:
                owner = self._owners.get(slot)
                if owner is not None:
                    owner.on_output(slot, data, flags)
            for fid, value in fres:
                fut = self._futures.pop(fid, None)
                if fut is not None and not fut.done():
                    fut.set_result(value)
            if self.engine.has_work():
                self._wake.set()


_TICKERS: Dict[int, Ticker] = {}


def ticker_for(engine) -> Ticker:
    loop = asyncio.get_running_loop()
    key = (id(loop), id(engine))
    t = _TICKERS.get(key)
    if t is None or t.loop.is_closed():
        t = Ticker(engine, loop)
        _TICKERS[key] = t
    return t
