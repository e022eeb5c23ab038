"""GPU: the native data plane with the CDNA4 HIP engine vs the FastAPI conformance app."""
import pytest

import test_native_server as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(T.SCENARIOS))
def test_native_hip_matches_python(name, monkeypatch):
    """HIP engine + verify mode: every stream and final is also checked against the
    shadow C++ CPU oracle inside the server (byte-identical or counted as mismatch)."""
    from quorum_amd.ops import native

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    T.test_native_matches_python(name)
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
    R.test_random_session_native_matches_python(seed)
    assert ext.server_counters()["verify_mismatches"] == before
