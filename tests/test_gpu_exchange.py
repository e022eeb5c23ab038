"""GPU: the exchange's RCCL bulk plane (ncclSend / ncclRecv rounds, HBM to HBM).

A 1-GPU box hosts a world-size-1 communicator (RCCL rejects two ranks on one device), so
the self-test sends every payload to itself: the mesh (loopback frames), rank 0's round
manifests, communicator formation (epoch), one ncclGroup per round with a send and a
receive to self, the staging receive and the device-to-device copy into the HBM sink —
then every byte is checked on the host.  Cross-rank behaviour is covered by the same code
over the TCP mesh (test_native_spread.py) and by bench.py's spread check in the driver's
multi-GPU runs."""
import pytest

from quorum_amd.ops import native

from live_upstream import free_port_block

pytestmark = pytest.mark.gpu


def test_rccl_bulk_rounds_loopback():
    ext = native.require()
    assert ext.device_count() > 0
    res = ext.exchange_selftest({"rank": 0, "world": 1, "transport": "rccl", "device": 0,
                                 "port": free_port_block(1), "timeout": 60.0}, 50)
    assert res["ok"], res
    assert res["epochs"] >= 1 and res["rccl_rounds"] >= 1 and res["mesh_finals"] == 0, res
    assert res["bulk"] == 50 and res["data"] == 50 and res["sent"] == 50, res
    print("rccl loopback: %d rounds, %.1f ms for 50 finals" % (res["rccl_rounds"], 1e3 * res["wall_s"]))


def test_tcp_exchange_loopback():
    ext = native.require()
    res = ext.exchange_selftest({"rank": 0, "world": 1, "transport": "tcp", "port": free_port_block(1)}, 50)
    assert res["ok"] and res["mesh_finals"] == 50 and res["rccl_rounds"] == 0, res
