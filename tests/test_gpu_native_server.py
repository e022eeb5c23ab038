"""GPU: the native data plane with the CDNA4 HIP engine vs the FastAPI conformance app."""
import pytest

import test_native_server as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tick_mode", ["loops", "lanes"])
@pytest.mark.parametrize("name", sorted(T.SCENARIOS))
def test_native_hip_matches_python(name, tick_mode, monkeypatch):
    """HIP engine + verify mode: every stream and final is also checked against the
    shadow C++ CPU oracle inside the server (byte-identical or counted as mismatch).
    loops: io loops post into the multi-door grid (the default); lanes: the shared engine."""
    from quorum_amd.ops import native

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    T.test_native_matches_python(name, tick_mode)
    assert ext.server_counters()["verify_mismatches"] == before


def test_native_hip_keepalive(monkeypatch):
    import live_upstream as L
    orig = L.native_server

    def hip_server(cfg, engine="cpu", threads=1, env_key=""):
        return orig(cfg, engine="hip", threads=threads, env_key=env_key)

    monkeypatch.setattr(T, "native_server", hip_server)
    T.test_native_keepalive_many_requests()


@pytest.mark.parametrize("seed", range(40))
def test_native_hip_random_sessions(seed, monkeypatch):
    """Random sessions (test_native_random_differential) through the HIP engine + verify."""
    from quorum_amd.ops import native

    import test_native_random_differential as R

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    R.run_random_session(seed, "loops" if seed % 2 else "lanes")
    assert ext.server_counters()["verify_mismatches"] == before


def test_gpu_bench_headline_valid(tmp_path):
    """The headline bench on the HIP engine (shared engine, pipelined tick lanes, persistent
    grids, result views) under full closed-loop load: every response is validated byte for
    byte by the load generator, so a lane that reuses an output arena too early, or any other
    cross-tick corruption, fails here."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QMX_BENCH_ENGINE="hip")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "4", "--warmup", "1",
                        "--batch", "8192", "--port", "23400"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=180)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert r.returncode == 0 and res["valid"] and res["invalid"] == 0, (res.get("invalid"), r.stderr[-2000:])
    assert res["validated"] == 4 * 8192 and res["breakdown_one_rank"]["kernel_launches"] > 0
