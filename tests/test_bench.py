"""bench.py contract (the driver's headline measurement): run from a foreign cwd, one JSON
line from rank 0 with the BASELINE.json metric and the required keys; world 2 through
``torch.distributed.run`` with the gloo backend on CPU (the MI355X node uses RCCL)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    """A bench base port below the ephemeral range: the bench also binds base + 7.. (mesh),
    base + 50.. (spread check) and base + 100.. (mocks)."""
    import random

    for _ in range(200):
        base = random.randrange(20000, 29000)
        try:
            for off in (0, 7, 8, 50, 57, 58, 100, 101, 110, 111):
                with socket.socket() as s:
                    s.bind(("127.0.0.1", base + off))
            return base
        except OSError:
            continue
    raise RuntimeError("no free port block")


def _env():
    e = dict(os.environ)
    e.pop("PYTHONPATH", None)  # the bench (and its workers) must find the package by themselves
    e["QMX_BENCH_ENGINE"] = "cpu"
    return e


def _check(line: str, n: int, steps: int, warmup: int):
    res = json.loads(line)
    assert KEYS <= set(res), KEYS - set(res)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert res["metric"] == base["metric"]
    assert res["n_gpus"] == n and res["steps"] == steps and res["warmup"] == warmup
    assert res["value"] > 0 and res["errors"] == 0
    assert res["scaling"] == "weak" and res["higher_is_better"] is True
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in res["config"]
    return res


def _json_lines(out: str):
    return [ln for ln in out.splitlines() if ln.startswith("{") and '"metric"' in ln]


def test_bench_single_rank_foreign_cwd(tmp_path):
    port = _free_port()
    r = subprocess.run([sys.executable, BENCH, "--steps", "2", "--warmup", "1", "--batch", "128", "--threads", "2",
                        "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = _check(lines[0], 1, 2, 1)
    assert res["config"]["global_batch"] == 128


@pytest.mark.slow
def test_bench_two_ranks_torchrun(tmp_path):
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH,
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "128", "--threads", "2",
                        "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = _check(lines[0], 2, 2, 1)
    assert res["config"]["global_batch"] == 256
    assert res["config"]["parallelism"].startswith("dp2")
    assert res["spread_check"]["ok"] is True, res["spread_check"]


@pytest.mark.slow
def test_bench_two_ranks_spread_check_failure_is_agreed(tmp_path):
    """One rank's spread check fails before its proxy starts: every rank still runs the same
    collectives (no rank left waiting in a barrier), the headline line is printed and valid,
    and the failure is reported under spread_check."""
    port = _free_port()
    env = dict(_env(), QMX_BENCH_SPREAD_FAIL_RANK="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH,
                        "--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "64", "--threads", "2",
                        "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    # the headline responses were fine: the run is valid, the failed spread check is reported
    # on its own (checks_ok false, a warning on stderr) instead of losing the measurement
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "post-timing check FAILED" in r.stderr
    res = _check(_json_lines(r.stdout)[0], 2, 1, 0)
    assert res["headline_valid"] is True and res["valid"] is True and res["checks_ok"] is False
    sc = res["spread_check"]
    assert sc["ok"] is False
    assert "injected" in sc["per_rank"][1]["error"] and "another rank's spread set failed" in sc["per_rank"][0]["error"]


@pytest.mark.slow
def test_bench_gpus_flag_self_launches_ranks(tmp_path):
    """``python bench.py --gpus 4`` with no launcher starts its own 4 ranks (a child
    torch.distributed.run): one JSON line, n_gpus 4, one breakdown row per rank scraped from
    that rank's own proxy (4 distinct pids), and a spread check whose rows carry each rank's
    own counters."""
    port = _free_port()
    env = dict(_env(), QMX_BENCH_NDEV="1")  # rehearsal: the ranks share (at most) one GPU
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "2", "--warmup", "1", "--batch", "128",
                        "--threads", "2", "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = _check(lines[0], 4, 2, 1)
    assert res["valid"] is True and res["config"]["global_batch"] == 512
    rows = res["breakdown_per_rank"]
    assert [x["rank"] for x in rows] == [0, 1, 2, 3]
    assert len({x["pid"] for x in rows}) == 4 and all(x["requests"] == 256 for x in rows)
    assert rows[0]["pid"] == res["breakdown_one_rank"]["pid"]
    sc = res["spread_check"]
    assert sc["ok"] is True and sc["requests"] == 4 * 2048 and sc["delta_mismatch"] == 0 and sc["invalid"] == 0
    # the production defaults: the short final texts ride the mesh behind their deltas
    assert sc["eager_finals"] == 4 * 2048 and sc["remote_ends"] == {"text": 4 * 2048}
    # the ranks share (no) GPU: the rendezvous set's final texts move in tcpbulk rounds — the
    # RCCL round protocol (announce, rank-0 manifests, epochs) with the socket executor
    assert sc["transport"] == "tcpbulk" and sc["bulk_formed"] is True
    assert sc["bulk_rounds"] > 0 and sc["mesh_finals"] == 0
    assert sc["rendezvous"]["remote_ends"] == {"text": 4 * 512}
    assert len({x["pid"] for x in sc["per_rank"]}) == 4
    # BASELINE config 3 after the spread check: aggregate4, spread, every remote final through
    # a bulk round (tcpbulk: the ranks share no GPU), every response validated
    c3 = res["config3"]
    assert c3["ok"] is True and c3["invalid"] == 0 and c3["requests"] == 4 * 4096 and c3["req_s"] > 0, c3
    assert c3["transport"] == "tcpbulk" and c3["bulk_rounds"] > 0 and c3["mesh_finals"] == 0, c3
    assert c3["delta_mismatch"] == 0 and "degraded" not in c3, c3
    # one-session latency probes, every response validated: the eager default, rendezvous
    # (every text through a round) and the same config placed locally
    assert None not in (sc["probe_p50_latency_ms"], sc["local_probe_p50_latency_ms"],
                        sc["rendezvous"]["probe_p50_latency_ms"])
    # (a rank's load generator connects to the shared port: any rank's proxy may own a
    # session, so the per-path counts are checked as totals)
    assert sum(r["main_probe"].get("eager_finals", 0) for r in sc["per_rank"]) == 4 * 256
    assert sum(r["main_probe"].get("bulk_rounds", 0) for r in sc["per_rank"]) == 0
    assert sum(r["rendezvous_probe"].get("bulk_rounds", 0) for r in sc["per_rank"]) > 0
    assert sc["hops_us_probe"]["last_delta_to_final"] is not None
    # every session has one remote stream, run by the next rank: each rank's own counter
    # is its own share, and the shares add up to every session once
    assert sum(x["main_load"]["remote_streams"] for x in sc["per_rank"]) == 4 * 2048
    assert all(0 < x["main_load"]["remote_streams"] < 4 * 2048 for x in sc["per_rank"])


def test_bench_refuses_world_mismatch(tmp_path):
    """Under a launcher, --gpus must name the launcher's world: a mismatch is refused
    before anything starts (exit 2), never measured as some other world."""
    env = dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_pin_rank_numa_plan(monkeypatch):
    """bench.pin_rank: ranks bound to their GPU's NUMA node (fake device properties and
    topology); skipped for one rank, rehearsals with more ranks than GPUs, and opt-out."""
    import importlib.util
    from types import SimpleNamespace

    from quorum_amd.parallel import topology

    spec = importlib.util.spec_from_file_location("qmx_bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    buses = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5]
    fake_torch = SimpleNamespace(cuda=SimpleNamespace(get_device_properties=lambda r: SimpleNamespace(
        pci_domain_id=0, pci_bus_id=buses[r], pci_device_id=0)))
    monkeypatch.setattr(topology, "pci_numa_node", lambda d, b, dev, f=0: 0 if b < 0x80 else 1)
    got = {}
    monkeypatch.setattr(topology, "plan_rank_cpus",
                        lambda nodes, allowed: [[r] for r in range(len(nodes))] if len(set(nodes)) == 2 else None)
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.setdefault("cpus", list(cpus)))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.delenv("QMX_BENCH_PIN", raising=False)
    # no L3 topology -> the node split (plan_rank_cpus)
    monkeypatch.setattr(topology, "llc_cpus", lambda node: 0)
    r = bench.pin_rank(fake_torch, 8, 5, 8)
    assert r["numa_nodes"] == [0, 0, 0, 0, 1, 1, 1, 1] and r["pinned"] and r["how"] == "node" and r["cpus"] == 1
    assert got.pop("cpus") == [5]
    # L3s known: whole L3s, the quota share rounded up (16 CPUs of a 128-CPU quota over 8 ranks)
    monkeypatch.setattr(topology, "llc_cpus", lambda node: 16)
    monkeypatch.setattr(bench, "available_cores", lambda: 128)
    seen = {}
    monkeypatch.setattr(topology, "rank_llc_cpus",
                        lambda nodes, rank, per, allowed: seen.setdefault("per", per) and list(range(64, 80)))
    r = bench.pin_rank(fake_torch, 8, 5, 8)
    assert r["how"] == "llc" and r["cpus"] == 16 and seen["per"] == 16 and got.pop("cpus") == list(range(64, 80))
    monkeypatch.setattr(bench, "available_cores", lambda: 256)  # no quota: at most two L3s per rank
    seen.clear()
    bench.pin_rank(fake_torch, 8, 5, 8)
    assert seen["per"] == 32
    got.clear()
    assert bench.pin_rank(fake_torch, 1, 0, 8) is None
    assert bench.pin_rank(fake_torch, 8, 0, 1) is None  # more ranks than GPUs
    monkeypatch.setenv("QMX_BENCH_PIN", "0")
    assert bench.pin_rank(fake_torch, 8, 0, 8) is None


def test_bench_fails_on_invalid_responses(tmp_path):
    """A proxy that drops one delta in 50 (QMX_FAULT_DROP_DELTA) must fail the bench: the
    load generator validates every response, so a broken engine cannot score."""
    port = _free_port()
    env = dict(_env(), QMX_FAULT_DROP_DELTA="50")
    r = subprocess.run([sys.executable, BENCH, "--steps", "1", "--warmup", "0", "--batch", "200", "--threads", "2",
                        "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 1, r.stdout[-2000:]
    res = json.loads(_json_lines(r.stdout)[0])
    assert res["invalid"] > 0 and res["valid"] is False
    assert "invalid response" in r.stderr


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/quorum"), reason="reference checkout not present")
def test_bench_reference_same_harness(tmp_path):
    """--impl reference: the unmodified upstream proxy (scratch copy) behind the same mocks,
    load generator and validator — its responses satisfy the same event contract."""
    port = _free_port()
    r = subprocess.run([sys.executable, BENCH, "--impl", "reference", "--steps", "1", "--warmup", "0", "--batch", "16",
                        "--conns", "4", "--port", str(port)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(_json_lines(r.stdout)[0])
    assert res["config"]["impl"] == "reference" and res["validated"] == 16 and res["invalid"] == 0
    assert res["vs_baseline"] is None


@pytest.mark.parametrize("impl", ["native", "reference"])
def test_bench_nonstream1_config1(tmp_path, impl):
    """BASELINE config 1 (1 mock backend, non-streaming, CPU): every JSON body validated
    (message, usage, "backend" key), for the native proxy and the unmodified reference under
    the same harness; the harness ceiling rides along."""
    if impl == "reference" and not os.path.isdir("/root/reference/src/quorum"):
        pytest.skip("reference checkout not present")
    port = _free_port()
    r = subprocess.run([sys.executable, BENCH, "--scenario", "nonstream1", "--impl", impl, "--steps", "1",
                        "--warmup", "0", "--batch", "16" if impl == "reference" else "400", "--threads", "2",
                        "--conns", "4", "--port", str(port), "--ceiling", "0.5"],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(_json_lines(r.stdout)[0])
    assert res["valid"] and res["invalid"] == 0 and res["validated"] == (16 if impl == "reference" else 400)
    assert res["config"]["engine"] == ("cpu" if impl == "native" else "reference")
    assert res["harness_ceiling_req_s"] > 0 and res["harness_ceiling"]["invalid"] == 0


def test_bench_direct_harness_ceiling(tmp_path):
    """--scenario direct: the load generator straight against a mock (no proxy), every
    content byte of the mock's stream validated."""
    port = _free_port()
    r = subprocess.run([sys.executable, BENCH, "--scenario", "direct", "--steps", "1", "--warmup", "0", "--batch",
                        "500", "--conns", "4", "--port", str(port)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(_json_lines(r.stdout)[0])
    assert res["valid"] and res["validated"] == 500 and res["config"]["impl"] == "none (no proxy)"
    assert res["breakdown_one_rank"]["cores_busy"]["proxy"] == 0.0


def test_breakdown_loop_tick_fields():
    """bench.breakdown on two synthetic /metrics scrapes: the loop-tick hops (calibrated
    clocks), S3's event paths per item and the shader clock come from summable counters (the
    io loops' engines add up in /metrics), means over the window between the scrapes."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("qmx_bench_mod2", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    m0 = {"qmx_kernel_launches": 10.0, "qmx_kernel_hop_ticks": 10.0, "qmx_kernel_post_seen_us": 15.0,
          "qmx_kernel_done_host_us": 100.0, "qmx_kernel_stage_items": 0.0, "qmx_kernel_clk_cycles": 0.0,
          "qmx_kernel_clk_us": 0.0, "qmx_tick_seconds_count": 10.0, "qmx_tick_seconds_sum": 5e-4}
    m1 = dict(m0, qmx_kernel_launches=110.0, qmx_kernel_hop_ticks=110.0, qmx_kernel_post_seen_us=165.0,
              qmx_kernel_done_host_us=1400.0, qmx_kernel_stage_items=40.0, qmx_kernel_s3_events=1080.0,
              qmx_kernel_s3_full_parses=0.0, qmx_kernel_s3_template_hits=960.0, qmx_kernel_s3_hole_hits=80.0,
              qmx_kernel_stage4_us=240.0, qmx_kernel_clk_cycles=2.4e6, qmx_kernel_clk_us=1000.0,
              qmx_tick_seconds_count=110.0, qmx_tick_seconds_sum=5.5e-3, qmx_kernel_clock_window_us=12.0,
              qmx_kernel_clock_windows=40.0)
    bd = bench.breakdown(m0, m1, 1.0)
    assert bd["tick_hops_us_avg"] == {"post_seen": 1.5, "done_host": 13.0, "clock_window": 0.3}
    assert bd["s3_per_item"] == {"events": 27.0, "full_parses": 0.0, "template_hits": 24.0, "hole_hits": 2.0}
    assert bd["stage_us_per_item"]["stage4_us"] == 6.0
    assert bd["shader_mhz"] == 2400.0
    assert bd["tick_wall_us_avg"] == 50.0


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4])
def test_bench_aggregate4_spread_finals_through_rounds(tmp_path, world):
    """BASELINE config 3 in the timed region: 4 backends, aggregate strategy, sessions sharded
    over the ranks AND each session's backend streams spread over them, with every remote
    final text moved by a bulk round (``--eager-bytes 0``: rank-0 manifests, then RCCL
    ncclSend/ncclRecv on a GPU node — here the tcpbulk executor, ranks sharing no GPU).
    Every response is validated; every rank ran rounds; no text fell back to the mesh; the
    owner finalized the merged sessions on its engine (finalize_host 0)."""
    port = _free_port()
    env = dict(_env(), QMX_BENCH_NDEV="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--scenario", "aggregate4", "--placement", "spread",
                        "--eager-bytes", "0", "--steps", "2", "--warmup", "1", "--batch", "128", "--threads", "2",
                        "--conns", "8", "--port", str(port)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads(_json_lines(r.stdout)[0])
    assert res["valid"] is True and res["invalid"] == 0 and res["n_gpus"] == world
    assert "ep%d" % world in res["config"]["parallelism"] and "TCPBULK" in res["config"]["parallelism"]
    for row in res["breakdown_per_rank"]:
        x = row["exchange"]
        assert x["remote_streams"] > 0 and x["bulk_rounds"] > 0 and x["round_us_avg"] > 0, row
        assert x["eager_finals"] == 0 and x["mesh_finals"] == 0, row
        assert x["delta_mismatch"] == 0 and x["worker_nodata"] == 0, row
        assert row["finalize_host"] == 0, row


def test_spread_and_config3_summaries_report_degraded_and_invariants():
    """The summaries never hide a broken invariant or a round protocol that did not run: a
    rendezvous set without bulk rounds is DEGRADED (its finals took the mesh, still
    validated), a delta mismatch fails its pass, and config3's node req/s divides the total
    by the slowest rank's wall."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    ok_pass = {"ok": True, "requests": 100, "invalid": 0, "p50_latency_ms": 1.0, "remote_streams": 100,
               "delta_mismatch": 0, "worker_nodata": 0, "bulk_rounds": 0, "finalize_host": 0,
               "remote_texts_staged": 100, "remote_texts_hbm": 0}
    row = {"ok": True, "transport": "rccl", "main": {"load": ok_pass, "probe": ok_pass},
           "rendezvous": {"load": ok_pass, "probe": ok_pass, "bulk_formed": False,
                          "degraded": "spread_rendezvous: bulk rounds did not run (formed False, rounds 0)"},
           "local": {"probe": ok_pass}}
    out = b.spread_summary([row, row])
    assert out["ok"] is True and out["degraded"] and "bulk rounds did not run" in out["degraded"][0]
    assert out["finalize_host"] == 0 and out["remote_texts_gpu"]["staged"] == 800
    c3 = b.config3_summary([{"ok": True, "transport": "rccl",
                             "load": dict(ok_pass, req_s=50.0, bulk_rounds=7, p50_ttft_ms=0.3)},
                            {"ok": True, "transport": "rccl",
                             "load": dict(ok_pass, req_s=25.0, bulk_rounds=5, p50_ttft_ms=0.5)}])
    assert c3["requests"] == 200 and c3["req_s"] == 50.0  # 200 requests / the slower rank's 4 s
    assert c3["bulk_rounds"] == 12 and c3["ok"] is True and "degraded" not in c3


def test_pin_single_specs(monkeypatch):
    """bench.pin_single (one rank): ``compact-smt`` takes the quota rounded up to whole L3s
    on the GPU's node, ``@N`` a given count, a cpulist exactly those CPUs (within the
    affinity set), ``none`` nothing; a set that would be every allowed CPU binds nothing."""
    import importlib.util

    from quorum_amd.parallel import topology

    spec = importlib.util.spec_from_file_location("qmx_bench_mod2", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    got = {}
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.__setitem__("cpus", list(cpus)))
    monkeypatch.setattr(topology, "llc_cpus", lambda node: 16)
    monkeypatch.setattr(topology, "cpu_busy", lambda: {})
    asked = {}

    def compact(n, node, allowed, smt=False, busy=None):
        asked.update(n=n, node=node, smt=smt)
        return list(range(64, 64 + n))

    monkeypatch.setattr(topology, "compact_cpus", compact)
    monkeypatch.setattr(bench, "available_cores", lambda: 12)
    monkeypatch.delenv("QMX_BENCH_CPUS", raising=False)
    r = bench.pin_single(None, 0)  # no GPU: node 0
    assert r["pinned"] and asked == {"n": 16, "node": 0, "smt": True} and got.pop("cpus") == list(range(64, 80))
    monkeypatch.setenv("QMX_BENCH_CPUS", "compact@8")
    r = bench.pin_single(None, 0)
    assert asked["n"] == 8 and not asked["smt"] and r["cpus"] == 8
    monkeypatch.setenv("QMX_BENCH_CPUS", "8-11,300")
    r = bench.pin_single(None, 0)
    assert got.pop("cpus") == [8, 9, 10, 11] and r["cpus"] == 4
    monkeypatch.setenv("QMX_BENCH_CPUS", "none")
    assert bench.pin_single(None, 0) is None
    monkeypatch.delenv("QMX_BENCH_CPUS")
    monkeypatch.setattr(bench, "available_cores", lambda: 256)  # the whole machine: nothing to gain
    assert bench.pin_single(None, 0)["pinned"] is False


def _fake_mi355x_node(root):
    """A copy of the sysfs an 8 x MI355X node shows: 2 sockets x 64 cores x 2 SMT (CPU c and
    c + 128 are siblings), 16 CCDs of 8 cores (one L3 each), GPUs 0-3 on NUMA node 0 and 4-7
    on node 1 (KFD nodes 2-9, their PCI functions' numa_node)."""
    node = root / "devices/system/node"
    for n in range(2):
        d = node / f"node{n}"
        d.mkdir(parents=True)
        d.joinpath("cpulist").write_text(f"{64 * n}-{64 * n + 63},{128 + 64 * n}-{128 + 64 * n + 63}\n")
    for c in range(256):
        core = c % 128
        t = root / f"devices/system/cpu/cpu{c}/topology"
        t.mkdir(parents=True)
        t.joinpath("physical_package_id").write_text(f"{core // 64}\n")
        t.joinpath("core_id").write_text(f"{core % 64}\n")
        k = core // 8
        l3 = root / f"devices/system/cpu/cpu{c}/cache/index3"
        l3.mkdir(parents=True)
        l3.joinpath("shared_cpu_list").write_text(f"{8 * k}-{8 * k + 7},{128 + 8 * k}-{128 + 8 * k + 7}\n")
    kfd = root / "class/kfd/kfd/topology/nodes"
    for n in range(10):
        d = kfd / str(n)
        d.mkdir(parents=True)
        if n < 2:
            d.joinpath("properties").write_text("simd_count 0\n")
            continue
        g = n - 2
        bus = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5][g]
        d.joinpath("properties").write_text(f"simd_count 1024\ndomain 0\nlocation_id {bus << 8}\n")
        p = root / f"bus/pci/devices/0000:{bus:02x}:00.0"
        p.mkdir(parents=True)
        p.joinpath("numa_node").write_text("0\n" if g < 4 else "1\n")


@pytest.mark.parametrize("quota", [128, 16])
def test_bench_plan_for_8_gpus(tmp_path, quota):
    """`bench.py --plan --gpus 8` on a fake 8-GPU node: what each rank runs and binds to,
    before the driver's scaling run (round-5 review: the 8-GPU plan was never printed).  With
    a 128-CPU quota every rank gets one CCD of its GPU's socket — 16 CPUs, disjoint, the
    one-GPU bench's own shape (8 io threads, 4 load-generator threads, 2 x 2 mock threads) —
    and the quota covers the harness.  With the one-GPU box's 16-CPU quota on the whole node,
    the plan says the curve would measure the quota (quota_bound), not the GPUs."""
    import json

    _fake_mi355x_node(tmp_path)
    env = dict(_env(), QMX_SYSFS_ROOT=str(tmp_path), QMX_BENCH_QUOTA=str(quota))
    r = subprocess.run([sys.executable, BENCH, "--plan", "--gpus", "8"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["world"] == 8 and plan["gpu_numa_nodes"] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert not plan["overlapping_sets"]
    ranks = plan["ranks"]
    for x in ranks:
        assert x["how"] == "llc" and x["cpus"] == 16 and x["l3s"] == 1, x
        lo = 0 if x["numa_node"] == 0 else 64  # the CCD is on the rank's GPU's socket
        assert lo <= x["first"] < lo + 64 and x["last"] >= 128, x
        assert x["mock_processes"] == 2 and x["mock_threads"] == 4
    if quota == 128:
        assert all(x["io_threads"] == 8 and x["loadgen_threads"] == 4 and x["busy_threads"] == 16 for x in ranks)
        assert not plan["quota_bound"] and plan["cpus_bound_total"] == 128
    else:
        assert all(x["io_threads"] == 2 for x in ranks)
        assert plan["quota_bound"] and plan["quota_needed_cpus"] > 100
