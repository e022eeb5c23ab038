"""GPU tests: loop ticks — engines that post into doors of one shared multi-door persistent
grid (``HipGrid``, the io loops' tick path) — vs the C++ CPU engine, byte for byte.

Covers several doors ticking concurrently from their own threads (each door's sub-grid runs
its engine's ticks; slot state, content arenas and templates are per engine), the host's idle
stop followed by a relaunch at the next post, and tiny tiles / content overflow on a door.
"""
import random
import threading
import time

import pytest

from quorum_amd.ops import native
from quorum_amd.ops.native import NativeEngine

import engine_harness as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    e = native.require()
    assert e.device_count() > 0, "no GPU visible"
    return e


def _case(seed, n_streams=6):
    rng = random.Random(seed)
    tags = ["think", "reason", "reasoning", "thought"]
    raw = [H.rand_stream(rng) for _ in range(n_streams)]
    streams = [H.split_random(rng, r, rng.choice([3, 17, 64, 400, 5000])) for r in raw]
    filt = [rng.random() < 0.8 for _ in raw]
    emit = [rng.random() < 0.8 for _ in raw]
    return tags, streams, filt, emit, rng.randint(0, 10**9)


def test_grid_doors_match_cpu(ext):
    grid = ext.HipGrid(0, 3, 4)
    tags = ["think", "reason", "reasoning", "thought"]
    engs = [NativeEngine("hip", tags, device=0, max_slots=256, grid=grid, door=d) for d in range(3)]
    for seed in range(12):
        tags_, streams, filt, emit, tseed = _case(seed)
        cpu = H.run_engine(NativeEngine("cpu", tags_), streams, filt, emit, random.Random(tseed))
        got = H.run_engine(engs[seed % 3], streams, filt, emit, random.Random(tseed))
        assert got == cpu, seed
    st = grid.stats()
    assert st["grid_doors"] == 3 and st["grid_launches"] >= 1
    grid.stop()


def test_grid_doors_concurrent_threads(ext):
    """Three doors ticked at once from three threads (the io loops' pattern): every door's
    results equal the CPU engine's."""
    grid = ext.HipGrid(0, 3, 4)
    tags = ["think", "reason", "reasoning", "thought"]
    engs = [NativeEngine("hip", tags, device=0, max_slots=256, grid=grid, door=d) for d in range(3)]
    errors = []

    def worker(d):
        try:
            for seed in range(100 + 10 * d, 106 + 10 * d):
                tags_, streams, filt, emit, tseed = _case(seed, 8)
                cpu = H.run_engine(NativeEngine("cpu", tags_), streams, filt, emit, random.Random(tseed))
                got = H.run_engine(engs[d], streams, filt, emit, random.Random(tseed))
                if got != cpu:
                    errors.append((d, seed))
        except Exception as e:  # noqa: BLE001
            errors.append((d, repr(e)))

    ts = [threading.Thread(target=worker, args=(d,)) for d in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    grid.stop()


def test_grid_two_doors_per_engine(ext):
    """An engine with two doors (two ticks in flight: buffer sets, kernel parameters and
    template tables per door) matches the CPU engine; both doors are used."""
    grid = ext.HipGrid(0, 4, 4)
    tags = ["think", "reason", "reasoning", "thought"]
    for seed in range(8):
        tags_, streams, filt, emit, tseed = _case(900 + seed, 10)
        cpu = H.run_engine(NativeEngine("cpu", tags_), streams, filt, emit, random.Random(tseed))
        eng = NativeEngine("hip", tags, device=0, max_slots=256, grid=grid, door=2 * (seed % 2), ndoors=2)
        got = H.run_engine(eng, streams, filt, emit, random.Random(tseed))
        assert got == cpu, seed
    grid.stop()


def test_grid_idle_stop_and_relaunch(ext):
    """The host stops an idle grid (stop ticks on every door) and the next post relaunches it
    from where each door's relay left off."""
    grid = ext.HipGrid(0, 2, 2, idle_ms=5)
    tags = ["think"]
    eng = NativeEngine("hip", tags, device=0, max_slots=64, grid=grid, door=1)
    for rnd in range(3):
        tags_, streams, filt, emit, tseed = _case(500 + rnd, 3)
        cpu = H.run_engine(NativeEngine("cpu", tags_), streams, filt, emit, random.Random(tseed))
        got = H.run_engine(NativeEngine("hip", tags_, device=0, max_slots=64, grid=grid, door=rnd % 2),
                           streams, filt, emit, random.Random(tseed))
        assert got == cpu
        time.sleep(0.02)
        grid.housekeep()  # idle > 5 ms: stopped
        assert grid.stats()["grid_stops"] >= rnd + 1
    assert grid.stats()["grid_launches"] >= 3
    del eng
    grid.stop()


def test_grid_small_tiles_and_overflow(ext):
    grid = ext.HipGrid(0, 2, 4)
    for seed in range(6):
        tags, streams, filt, emit, tseed = _case(700 + seed, 5)
        cpu = H.run_engine(NativeEngine("cpu", tags), streams, filt, emit, random.Random(tseed))
        kw = {"tile_bytes": 1024} if seed % 2 else {"content_cap": 64}
        got = H.run_engine(NativeEngine("hip", tags, device=0, max_slots=64, grid=grid, door=seed % 2, **kw),
                           streams, filt, emit, random.Random(tseed))
        assert got == cpu, seed
    grid.stop()
