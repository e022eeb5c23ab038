"""GPU: the RCCL exchange transport (ncclAllGather on a dedicated HIP stream).

A 1-GPU box can only host a world-size-1 communicator (RCCL rejects two ranks on one
device), which still runs the whole transport: unique-id publication, communicator init,
the fixed-slot all-gather, the padded second phase for large payloads, D2H + parsing.
Cross-rank behaviour is covered by the same code under the TCP hub (test_native_spread.py)
and by the driver's 8-GPU runs."""
import os

import pytest

from quorum_amd.ops import native

pytestmark = pytest.mark.gpu


def test_rccl_transport_selftest(tmp_path):
    ext = native.require()
    assert ext.device_count() > 0
    res = ext.exchange_selftest({"rank": 0, "world": 1, "transport": "rccl", "device": 0,
                                 "id_file": str(tmp_path / "rccl.id")}, 100)
    assert res["ok"], res
    assert os.path.exists(tmp_path / "rccl.id")
    print("rccl round latency (us):", res["small_round_us"], res["large_round_us"])
