"""Process-level behaviour of the native data plane (no GPU):

* the kernel's fd table is grown once at start, before any io loop runs (``presize_fd_table``,
  qmx_server.cpp): growing it while serving waits out an RCU grace period in every thread
  that allocates an fd (measured on the MI355X box: io loops parked 70-210 ms in
  ``expand_files``, ``profiles/r6/stalls``);
* the soft fd limit is raised toward the hard one (a proxy holds clients + upstreams + pools);
* io-loop threads are named ``qmx-loop-N`` (``top -H``, the stall watchdog's dump);
* the bench's resident-memory probe (``bench.rss_mb``) reads /proc.
"""
import os
import resource
import sys

import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel
from live_upstream import native_server

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fdsize() -> int:
    for ln in open("/proc/self/status"):
        if ln.startswith("FDSize:"):
            return int(ln.split()[1])
    return 0


def _thread_names():
    names = []
    for t in os.listdir("/proc/self/task"):
        try:
            names.append(open(f"/proc/self/task/{t}/comm").read().strip())
        except OSError:
            pass
    return names


def test_server_presizes_fd_table_and_names_loop_threads():
    soft0, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    with native_server(cfg_parallel(2), threads=3):
        soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
        cap = (1 << 17) if hard == resource.RLIM_INFINITY else min(hard, 1 << 17)
        assert soft == (soft0 if soft0 >= cap else cap)
        if soft > 1024:
            # the table covers the whole limit now: no growth while serving
            assert _fdsize() >= min(soft, 1 << 17)
        names = _thread_names()
        for i in range(3):
            assert f"qmx-loop-{i}" in names, names


def test_bench_rss_probe():
    sys.path.insert(0, ROOT)
    import bench

    r = bench.rss_mb(os.getpid())
    assert r["VmRSS"] > 0 and r["VmHWM"] >= r["VmRSS"]
    assert bench.rss_mb(2 ** 22 + 12345) == {}  # no such process: nothing, no exception
