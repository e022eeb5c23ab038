"""GPU: persistent tick mode (the default; QMX_PERSISTENT=0 launches per tick) — one
long-lived grid per lane, ticks posted through a host-mapped doorbell instead of a launch
each (qmx_hip.hip qmx_tick_persistent).

Every result must equal the C++ CPU engine's, as in one-shot mode, including ticks with more
items than the grid has workgroups (a workgroup loops over items), fused finalize work,
two lanes with a grid each, and a grid that idled out and was relaunched."""
import random
import time

import pytest

from quorum_amd.ops import native
from quorum_amd.ops.native import NativeEngine

import engine_harness as H

pytestmark = pytest.mark.gpu


@pytest.fixture
def persistent(monkeypatch):
    e = native.require()
    assert e.device_count() > 0, "no GPU visible"
    monkeypatch.setenv("QMX_PERSISTENT", "1")
    monkeypatch.setenv("QMX_PERSISTENT_WG", "16")  # small grid: ticks with more items than workgroups
    return e


def _check(seed, n_streams, **kw):
    rng = random.Random(seed)
    tags = rng.sample(["think", "reason", "reasoning", "thought"], rng.randint(1, 3))
    raw = [H.rand_stream(rng) for _ in range(n_streams)]
    streams = [H.split_random(rng, r, rng.choice([5, 40, 400, 5000])) for r in raw]
    filt = [rng.random() < 0.8 for _ in raw]
    emit = [rng.random() < 0.8 for _ in raw]
    tseed = rng.randint(0, 10**9)
    cpu = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(tseed), **kw)
    eng = NativeEngine("hip", tags, device=0)
    hip = H.run_engine(eng, streams, filt, emit, random.Random(tseed), **kw)
    assert cpu == hip
    return eng._e.kernel_stats()


@pytest.mark.parametrize("seed", range(8))
def test_persistent_matches_cpu(persistent, seed):
    st = _check(8100 + seed, 40)
    assert st["persistent_grids"] >= 1 and st["persistent_ticks"] == st["launches"], st
    assert st["poll_fallbacks"] == 0, st


def test_persistent_wide_ticks_and_finalize(persistent):
    st = _check(8200, 200, strip_final=True, joiner="\n--\n")
    assert st["persistent_ticks"] >= 1 and st["fin_items"] >= 1 and st["poll_fallbacks"] == 0, st


def test_persistent_idle_exit_and_relaunch(persistent, monkeypatch):
    monkeypatch.setenv("QMX_PERSISTENT_IDLE_MS", "10")
    eng = NativeEngine("hip", ["think"], device=0)
    slot = eng.open(0, True, True)
    got = []
    for i in range(3):
        eng.feed(slot, H.event_bytes(random.Random(i), f"part{i} <think>x</think>"))
        res, _ = eng.tick(H.CREATED)
        got += [r[1] for r in res if r[0] == slot]
        time.sleep(0.05)  # longer than the grid's idle limit: it exits, the next tick relaunches
    eng.finish(slot)
    eng.tick(H.CREATED)
    assert eng.text(slot) == "part0 part1 part2 "
    st = eng._e.kernel_stats()
    assert st["persistent_grids"] >= 3 and st["poll_fallbacks"] == 0, st
    eng.release(slot)


def test_persistent_two_lanes(persistent):
    """Two lanes, a grid each, alternately driven by one thread: same bytes as the CPU engine."""
    rng = random.Random(8300)
    tags = ["think"]
    raw = [H.rand_stream(rng) for _ in range(24)]
    streams = [H.split_random(rng, r, 60) for r in raw]
    n = len(streams)
    cpu = H.run_engine(NativeEngine("cpu", tags), streams, [True] * n, [True] * n, random.Random(2))
    eng = NativeEngine("hip", tags, device=0, lanes=2)
    slots = [eng.open(i % 7, True, True) for i in range(n)]  # the harness's backend indices
    out = {s: b"" for s in slots}
    cur = [0] * n
    lane = 0
    while any(c <= len(s) for c, s in zip(cur, streams)) or eng.has_work():
        for i, chunks in enumerate(streams):
            if cur[i] < len(chunks):
                eng.feed(slots[i], chunks[cur[i]])
            elif cur[i] == len(chunks):
                eng.finish(slots[i])
            cur[i] += 1
        res, _f, taken = eng._e.tick_unsettled(H.CREATED, lane)
        for slot, data, _fl in res:
            out[slot] += data
        eng._e.settle(taken)
        lane ^= 1
    for i, s in enumerate(slots):
        assert out[s] == cpu[0][i][0], i
    st = eng._e.kernel_stats()
    assert st["persistent_grids"] >= 2 and st["poll_fallbacks"] == 0, st


@pytest.mark.parametrize("seed", range(4))
def test_oneshot_mode_matches_cpu(monkeypatch, seed):
    """QMX_PERSISTENT=0: the launch-per-tick path stays exact (rocprof kernel stats and the
    stage-timing benchmark use it)."""
    e = native.require()
    assert e.device_count() > 0
    monkeypatch.setenv("QMX_PERSISTENT", "0")
    st = _check(8400 + seed, 30)
    assert st["persistent_grids"] == 0 and st["launches"] >= 1 and st["poll_fallbacks"] == 0, st
