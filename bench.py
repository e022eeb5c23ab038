#!/usr/bin/env python3
"""Headline benchmark: proxied req/s (whole node) + p50 TTFT, 2-backend concatenate stream.

BASELINE.json metric/config: 2 mock backends, streaming ``concatenate`` with
``hide_intermediate_think: true`` and ``skip_final_aggregation: true``; every upstream
response is the survey's shape (role + 4 split <think> fragments + 20 tokens + stop +
[DONE]).  One rank per GPU (``torch.distributed.run``); each rank runs:

* its proxy (``--impl native``: C++ epoll data plane; ``python``: FastAPI/uvicorn workers)
  on ONE node-wide SO_REUSEPORT port — the kernel shards client sessions across the
  node's GPUs — with the CDNA4 tick kernel on its own GPU (``--engine hip``);
* two C++ mock backends and a C++ closed-loop load generator (synthetic traffic).

A *step* = ``--batch`` completed client requests per rank.  W warmup steps, then EXACTLY
K timed steps bracketed by barrier + ``torch.cuda.synchronize()``; the slowest rank's
time is used; rank 0 prints one JSON line.  ``value`` = total completed requests / time
(whole node).  Weak scaling: per-rank load is fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# BASELINE.md "same harness" rows: the unmodified reference proxy measured on the MI355X box
# by this bench (--impl reference: same C++ mocks, load generator, validator, 16 clients;
# profiles/r2/reference_same_harness_*.json).  Scenarios without such a row fall back to the
# survey's 8-vCPU container numbers and say so in the JSON line.
BASELINE_SOURCE_SAME = "reference proxy, same box + same harness (bench.py --impl reference)"
BASELINE_SOURCE_SURVEY = "reference proxy, survey container (8 vCPU, Python harness; SURVEY §6)"

# port layout above --port: +7.. exchange mesh, +50 the spread check's proxies (+57.. its mesh;
# +20 / +80 its rendezvous / local sets), +60 the config-3 pass (+67.. its mesh; sets run one at a time),
# +100 + 10 rank + i mock backends, +200 + rank / +230 + rank each rank's own admin port
# (headline / spread check)
ADMIN_OFF, SPREAD_ADMIN_OFF, LOCAL_ADMIN_OFF, RDV_ADMIN_OFF, C3_ADMIN_OFF = 200, 230, 240, 250, 260
RANK_PORT_OFF = 300  # multi-rank: rank r's proxy and load generator on port + 300 + r (QMX_BENCH_RANK_PORTS)
CONFIG3_REQUESTS = 4096  # per rank: the config-3 pass after the headline (spread, RCCL rounds)
PROBE_REQUESTS = 256  # spread check: requests of the one-connection latency probes

# BASELINE.json configs.  "headline" is the driver's metric; the others are measured with
# --scenario; every one with a reference number has it from the same harness.
SCENARIOS = {
    # headline: 131072 requests per step per rank, so the driver's 20 timed steps are one
    # load-generator run of >= 10 s on one GPU (~230k req/s): box noise, connection set-up and
    # drain are amortised (r2's 16384 gave a 1.4 s window that moved +-15% run to run)
    "headline": dict(n=2, strategy="concatenate", hide_final=False, skip=True, faults={}, timeout=30,
                     batch=131072, baseline=21.071, baseline_ttft_ms=619.6, baseline_source=BASELINE_SOURCE_SAME,
                     desc="2 mock backends, streaming concatenate, hide_intermediate_think"),
    "aggregate4": dict(n=4, strategy="aggregate", hide_final=False, skip=False, faults={}, timeout=30,
                       baseline=10.09, baseline_ttft_ms=1191.9, baseline_source=BASELINE_SOURCE_SAME,
                       desc="4 mock backends, streaming aggregate strategy (LLM4 also aggregates)"),
    "highqps8": dict(n=8, strategy="concatenate", hide_final=True, skip=True, faults={}, timeout=30,
                     baseline=6.695, baseline_ttft_ms=2183.2, baseline_source=BASELINE_SOURCE_SAME,
                     desc="8 mock backends, streaming, hide_final_think + skip_final_aggregation"),
    "failure": dict(n=2, strategy="concatenate", hide_final=False, skip=False, timeout=2,
                    faults={1: ["--fail-rate", "0.3", "--drop-rate", "0.2", "--null-rate", "0.1"]},
                    baseline=21.14, baseline_ttft_ms=620.5, baseline_source=BASELINE_SOURCE_SAME,
                    desc="2 mock backends, backend 2 injects 30% HTTP 500 / 20% mid-stream "
                                       "disconnect / 10% content:null; 2 s timeout"),
    # config 5 as round 4 measured it: the faulty backend writes each event on its own (a
    # trickling upstream: a receive and a tick per event); "failure" writes a response at once
    "failure_trickle": dict(n=2, strategy="concatenate", hide_final=False, skip=False, timeout=2,
                            faults={1: ["--fail-rate", "0.3", "--drop-rate", "0.2", "--null-rate", "0.1",
                                        "--trickle", "1"]},
                            baseline=21.14, baseline_ttft_ms=620.5, baseline_source=BASELINE_SOURCE_SAME,
                            desc="config 5 with the faulty backend trickling its events (one write each)"),
    # the headline with per-token upstreams: both backends write every SSE event on its own,
    # with no delay (a real LLM server flushes one event per token) — a receive and an engine
    # feed per event instead of one per response.  The reference buffers whole bodies, so the
    # write granularity does not change its work: its headline number is the baseline.
    "trickle": dict(n=2, strategy="concatenate", hide_final=False, skip=True, faults={}, timeout=30,
                    mock_args=["--trickle", "1"], baseline=21.071, baseline_ttft_ms=619.6,
                    baseline_source=BASELINE_SOURCE_SAME,
                    desc="2 mock backends writing each SSE event on its own (per-token upstream writes), "
                         "streaming concatenate, hide_intermediate_think"),
    # steady-state serving shape: backends pace their events (10 ms apart, like a decoding
    # LLM), many concurrent sessions, each tick sees a few events of many streams.  TTFT is
    # bounded below by the mock's own first-content time (5 events x 10 ms = 50 ms).
    # BASELINE config 1: 1 mock backend, non-streaming, the C++ CPU engine (no GPU work: one
    # valid backend is quorum's passthrough, oai_proxy.py:1130-1137, 1356-1380 — the upstream
    # JSON plus "backend": name; the load generator checks message content, usage and that key)
    "nonstream1": dict(n=1, strategy="concatenate", hide_final=False, skip=False, faults={}, timeout=30,
                       stream=False, engine="cpu", baseline=56.647, baseline_ttft_ms=282.2,
                       baseline_source=BASELINE_SOURCE_SAME,
                       desc="1 mock backend, non-streaming concatenate (passthrough), CPU engine"),
    # the harness alone: the load generator straight against one mock backend, no proxy, same
    # validation (every content byte of the mock's stream) — SURVEY §6 row 1 / §7.4 item 4.
    # Every other scenario also measures this after its timed region (harness_ceiling).
    "direct": dict(n=1, strategy="concatenate", hide_final=False, skip=True, faults={}, timeout=30, direct=True,
                   batch=131072, baseline=319.0, baseline_ttft_ms=18.9, baseline_source="direct mock backend under the "
                   "survey's Python harness (SURVEY §6 row 1: the harness ceiling there)",
                   desc="harness ceiling: load generator -> 1 mock backend, no proxy"),
    "paced": dict(n=2, strategy="concatenate", hide_final=False, skip=True, faults={}, timeout=30,
                  mock_args=["--delay-us", "10000"], conns=1024, baseline=None,
                  desc="2 mock backends pacing events 10 ms apart (first content at 50 ms), 1024 sessions "
                       "in flight, streaming concatenate + hide_intermediate_think"),
}


def _gpu_held() -> bool:
    """Does this process hold the GPU (a KFD process entry or an open device file)?"""
    if os.path.exists(f"/sys/class/kfd/kfd/proc/{os.getpid()}"):
        return True
    try:
        for fd in os.listdir("/proc/self/fd"):
            t = os.readlink(f"/proc/self/fd/{fd}")
            if t == "/dev/kfd" or t.startswith("/dev/dri/"):
                return True
    except OSError:
        pass
    return False


def _trace(stage: str) -> None:
    if os.environ.get("QMX_BENCH_FDTRACE"):
        print(f"bench rank {os.environ.get('RANK', '0')}: {stage}: gpu held {_gpu_held()}", file=sys.stderr, flush=True)


def _barrier(dist, on_gpu: bool) -> None:
    """dist.barrier(), but a rehearsal's gloo group synchronises with a CPU all-reduce:
    gloo's barrier() touches the CUDA device (it picks a device for its work), and a box
    counts every process holding the GPU."""
    if on_gpu:
        dist.barrier()
    else:
        import torch

        dist.all_reduce(torch.zeros(1))


def _trace_watch() -> None:
    """QMX_BENCH_FDTRACE: report the main thread's stack when this process first holds the GPU."""
    if not os.environ.get("QMX_BENCH_FDTRACE"):
        return
    import threading
    import traceback

    main = threading.main_thread().ident

    def watch():
        while not _gpu_held():
            time.sleep(0.05)
        fr = sys._current_frames().get(main)
        print(f"bench rank {os.environ.get('RANK', '0')}: GPU first held at:\n" + "".join(traceback.format_stack(fr)),
              file=sys.stderr, flush=True)

    threading.Thread(target=watch, daemon=True).start()


def _kill(procs):
    for p in procs:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except OSError:
            pass
    for p in procs:
        try:
            p.wait(timeout=10)
        except Exception:  # noqa: BLE001
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass


def available_cores() -> int:
    """CPU cores this job may use: the cgroup CPU quota if one is set, else the affinity set
    (``nproc`` on a GPU box shows the whole machine)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def pin_rank(torch, world: int, local_rank: int, n_dev: int):
    """One rank per GPU: bind this rank (and the proxy, mocks and load generator it spawns) to
    a compact CPU set on its GPU's NUMA node — whole L3s, both SMT threads, its share of the
    job's CPU quota rounded up to whole L3s and at most two (one rank measured the same on one
    or two CCDs and slower spread further: profiles/r5/pinning), ranks sharing a node on
    consecutive L3s (parallel/topology.py rank_llc_cpus); where that does not fit, the node's
    cores split between its ranks (rank_cpus).  Skipped for one rank (pin_single), for
    rehearsals with more ranks than GPUs, when NUMA information is missing, and with
    QMX_BENCH_PIN=0."""
    if world <= 1 or n_dev == 0 or os.environ.get("QMX_BENCH_PIN", "1") == "0":
        return None
    from quorum_amd.parallel.topology import llc_cpus, pci_numa_node, plan_rank_cpus, rank_llc_cpus

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    rehearse = os.environ.get("QMX_BENCH_PIN_REHEARSE") == "1"  # ranks sharing GPU 0, bound as if on its node
    if n_dev < local_world and not rehearse:
        return None
    nodes = []
    if n_dev < local_world:  # rehearsal: every rank on GPU 0's node (KFD topology: no HIP call here)
        from quorum_amd.parallel.topology import gpu_numa_nodes

        g = gpu_numa_nodes()
        nodes = [max(0, g[0]) if g else 0] * local_world
    for r in range(len(nodes), local_world):
        pr = torch.cuda.get_device_properties(r)
        nodes.append(pci_numa_node(pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))
    allowed = sorted(os.sched_getaffinity(0))
    cpus, how = rank_cpu_set(nodes, local_rank, allowed, available_cores())
    if not cpus:
        return {"numa_nodes": nodes, "pinned": False}
    os.sched_setaffinity(0, cpus)
    return {"numa_nodes": nodes, "pinned": True, "how": how, "cpus": len(cpus), "first": cpus[0], "last": cpus[-1]}


def rank_cpu_set(nodes, local_rank: int, allowed, quota: int):
    """(CPUs, how) a rank binds to (pin_rank; nothing is bound here): whole L3s of its GPU's
    NUMA node, its share of the quota rounded up to whole L3s and at most two ("llc"); else
    the node's cores split between its ranks ("node"); else (None, None)."""
    from quorum_amd.parallel.topology import llc_cpus, plan_rank_cpus, rank_llc_cpus

    llc = llc_cpus(max(0, nodes[local_rank]))  # 0: no cache topology -> the node split
    if llc > 0:
        share = max(1, quota // max(1, len(nodes)))
        per_rank = min(-(-share // llc) * llc, 2 * llc)
        # every rank decides alone: whole L3s only if EVERY rank of the node gets its own, or
        # a rank that got L3s would overlap the ones that fell back to the node split
        sets = [rank_llc_cpus(nodes, r, per_rank, allowed) for r in range(len(nodes))]
        if all(sets):
            return sets[local_rank], "llc"
    plan = plan_rank_cpus(nodes, allowed)
    if plan and plan[local_rank]:
        return plan[local_rank], "node"
    return None, None


# Cores one rank's harness keeps busy at the headline's full rate on the MI355X box (proxy
# 6.8, mocks 3.0, load generator 3.3: profiles/r6/engine_ab/bench_1.json `cores_busy`)
HEADLINE_CORES_PER_RANK = 13.1


def node_plan(world: int, sc: dict, args, quota: int, allowed, nodes) -> dict:
    """What `bench.py --gpus world` will run on this node, per rank, without running it:
    io threads, load-generator and mock threads, the CPU set and L3s each rank binds to, and
    whether the job's CPU quota can feed `world` ranks at the one-GPU rate.  Every rank's
    proxy, mocks and load generator share its CPU set, so a quota below world x
    HEADLINE_CORES_PER_RANK makes the scaling curve measure the quota, not the GPUs."""
    from quorum_amd.parallel.topology import _llc_key

    threads = args.threads if args.threads > 0 else max(2, min(8, quota // (2 * world)))
    ranks = []
    seen, overlap = set(), False
    for r in range(world):
        cpus, how = rank_cpu_set(nodes, r, allowed, quota) if world > 1 else (None, None)
        overlap = overlap or bool(seen & set(cpus or []))
        seen |= set(cpus or [])
        lg = args.lg_threads if args.lg_threads > 0 else (4 if cpus else 3)
        mock = sc["n"] * args.mock_threads
        l3s = sorted({_llc_key(c, __import__("quorum_amd.parallel.topology", fromlist=["x"]).CPU_DEVICES)
                      for c in (cpus or [])})
        ranks.append({"rank": r, "numa_node": nodes[r], "io_threads": threads, "loadgen_threads": lg,
                      "mock_processes": sc["n"], "mock_threads": mock, "busy_threads": threads + lg + mock,
                      "cpus": len(cpus) if cpus else None, "first": cpus[0] if cpus else None,
                      "last": cpus[-1] if cpus else None, "l3s": len(l3s) if cpus else None, "how": how})
    bound = sum(x["cpus"] or 0 for x in ranks)
    demand = round(HEADLINE_CORES_PER_RANK * world, 1)
    return {"world": world, "quota_cpus": quota, "allowed_cpus": len(allowed), "gpu_numa_nodes": nodes,
            "ranks": ranks, "cpus_bound_total": bound,
            "headline_cores_demand": demand,
            # the curve measures GPUs only while the quota covers every rank's harness
            "quota_bound": quota < demand,
            "quota_needed_cpus": int(-(-demand // 1)),
            "overlapping_sets": overlap}


def pin_single(torch, n_dev: int):
    """One rank: bind the bench — proxy, mocks and load generator inherit it — to a compact CPU
    set on the GPU's NUMA node (QMX_BENCH_CPUS, default ``compact-smt``):

    * ``compact-smt``: both hardware threads of as many physical cores as the job's CPU quota
      needs, rounded up to whole last-level caches (on the MI355X box: a quota of 16 CPUs =
      one 8-core CCD), the least-loaded L3s first (a 0.2 s /proc/stat sample: the host is
      shared with other jobs).  The proxy and its loopback peers then share one L3
      instead of wherever the scheduler scatters them over a 256-thread machine: headline
      365-381k req/s against 268-298k unbound, proxy CPU 17.4 vs 22-25 us per request
      (profiles/r5/pinning).  Partial CCDs measured slower (`compact-smt@24`: 223k);
    * ``compact`` / ``compact-smt@N``: one thread per core / N CPUs;
    * a cpulist (``64-79``): exactly those; ``none``: no binding."""
    spec = os.environ.get("QMX_BENCH_CPUS", "compact-smt")
    if not spec or spec == "none":
        return None
    from quorum_amd.parallel.topology import compact_cpus, cpu_busy, llc_cpus, parse_cpulist, pci_numa_node

    allowed = sorted(os.sched_getaffinity(0))
    if spec.startswith("compact"):
        node = 0
        if n_dev:
            pr = torch.cuda.get_device_properties(0)
            node = max(0, pci_numa_node(pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))
        kind, _, n = spec.partition("@")  # compact[-smt][@N CPUs]
        if n:
            want = int(n)
        else:  # the quota, rounded up to whole last-level caches
            llc = max(1, llc_cpus(node))
            want = -(-available_cores() // llc) * llc
        if want >= len(allowed):
            return {"pinned": False, "spec": spec, "reason": "the set would be every allowed CPU"}
        # the least-loaded L3s of the node (the host's other tenants), packed
        cpus = compact_cpus(want, node, allowed, smt=kind == "compact-smt", busy=cpu_busy())
    else:
        cpus = [c for c in parse_cpulist(spec) if c in set(allowed)]
    if not cpus:
        return {"pinned": False, "spec": spec}
    os.sched_setaffinity(0, cpus)
    return {"pinned": True, "spec": spec, "cpus": len(cpus), "first": cpus[0], "last": cpus[-1]}


def write_config(path: str, mock_ports, skip_final: bool, tile: int, sc=None, placement="local") -> None:
    import yaml

    sc = sc or SCENARIOS["headline"]
    block = {"separator": "\n-------------\n", "hide_intermediate_think": True,
             "hide_final_think": bool(sc["hide_final"]), "thinking_tags": ["think", "reason", "reasoning", "thought"],
             "skip_final_aggregation": skip_final}
    cfg = {
        "settings": {"timeout": sc["timeout"]},
        "primary_backends": [{"name": f"LLM{i + 1}", "url": f"http://127.0.0.1:{p}/v1", "model": f"mock-{i + 1}"}
                             for i, p in enumerate(mock_ports)],
        "iterations": {"aggregation": {"strategy": sc["strategy"]}},
        "strategy": {"concatenate": block},
        "runtime": {"tile_bytes": tile, "max_slots": 4096, "content_cap": 1 << 18, "placement": placement},
    }
    if sc["strategy"] == "aggregate":
        cfg["strategy"]["aggregate"] = dict(block, aggregator_backend=f"LLM{len(mock_ports)}",
                                            intermediate_separator="\n\n---\n\n", include_source_names=True,
                                            source_label_format="Response from {backend_name}:\n",
                                            prompt_template="Synthesize:\n\n{responses}",
                                            include_original_query=True)
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)


def mock_expected(bin_dir) -> dict:
    """What a client must see from one mock backend (qmx_mock --print-expected): the streamed
    content outside the think block, and the non-streaming message content."""
    out = subprocess.run([os.path.join(bin_dir, "qmx_mock"), "--print-expected", "1", "--tokens", "20", "--think", "1"],
                         capture_output=True, text=True, timeout=30, check=True)
    return json.loads(out.stdout)


def expect_spec(path: str, sc: dict, skip_final: bool, exp: dict, path_prefix: str = "chatcmpl-parallel") -> None:
    """Write qmx_loadgen's --expect file for a scenario: the exact event contract every
    response must satisfy (role first, [DONE] last, per-backend content, final event)."""
    if sc.get("direct"):  # the mock's own stream: every content byte, its role / stop events skipped
        lines = ["role 0", "done 1", "empty allowed", f"stream chatcmpl-mock exact {exp['raw_text'].encode().hex()}",
                 "final absent", "error absent"]
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return
    if not sc.get("stream", True):
        if sc["n"] != 1:
            raise ValueError("non-streaming bench scenarios are single-backend (passthrough)")
        u = exp["usage"]
        lines = ["json 1", f"message {exp['message'].encode().hex()}", f"usage {u[0]} {u[1]} {u[2]}",
                 f"field backend {'LLM1'.encode().hex()}"]
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return
    sep = "\n" + "\n-------------\n"  # streaming final joiner: "\n" + separator (oai_proxy.py:834-841)
    text = exp["stream_text"]
    faulty = set(sc["faults"])
    lines = ["role 1", "done 1"]
    for i in range(sc["n"]):
        mode = "prefix" if i in faulty else "exact"
        lines.append(f"stream {path_prefix}-{i} {mode} {text.encode().hex()}")
    if skip_final:
        lines.append("final absent")
    elif sc["strategy"] == "aggregate":
        lines.append("final any " + exp["message"].encode().hex())  # the aggregator's answer, verbatim
    else:
        good = [i for i in range(sc["n"]) if i not in faulty]
        opts = {sep.join([text] * len(good))}
        if faulty:  # a faulty backend contributes its text only when its stream succeeded
            opts.add(sep.join([text] * (len(good) + len(faulty))))
        lines.append("final any " + " ".join(sorted(o.encode().hex() for o in opts)))
    lines.append("error absent")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def loadgen(bin_dir, port, conns, requests, threads, timeout, expect=None, path="/v1/chat/completions", stream=True):
    cmd = [os.path.join(bin_dir, "qmx_loadgen"), "--port", str(port), "--conns", str(conns),
           "--requests", str(requests), "--threads", str(threads), "--timeout", str(timeout),
           "--path", path, "--stream", "1" if stream else "0"]
    if expect:
        cmd += ["--expect", expect]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 60)
    if out.returncode != 0:
        raise RuntimeError(f"loadgen failed: {out.stderr}")
    if out.stderr.strip():
        print(out.stderr.strip()[-3000:], file=sys.stderr, flush=True)  # the first invalid responses
    return json.loads(out.stdout.strip().splitlines()[-1])


def wait_port(host: str, port: int, timeout: float) -> bool:
    """A TCP listener answers on host:port (the direct check's mock: no /health route)."""
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            with socket.create_connection((host, port), timeout=1):
                return True
        except OSError:
            time.sleep(0.05)
    return False


def harness_ceiling(bin_dir, mock_port, args, mock_proc, tmp) -> dict:
    """The load generator straight against one mock backend for ``args.ceiling`` seconds, with
    the bench's connections, threads and validation (every content byte of the mock's stream):
    what the harness alone sustains on this box, next to the proxied number."""
    import resource

    spec = os.path.join(tmp, "expect_direct.txt")
    expect_spec(spec, SCENARIOS["direct"], True, mock_expected(bin_dir))
    ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    m0 = cpu_seconds(mock_proc.pid)
    st = loadgen(bin_dir, mock_port, args.conns, 10**9, args.lg_threads, args.ceiling, spec)
    ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    el = max(st["elapsed_s"], 1e-9)
    return {"req_s": round(st["completed"] / el, 1), "seconds": round(el, 3), "completed": st["completed"],
            "invalid": st["invalid"], "errors": st["errors"] + st["non200"], "p50_ttft_ms": st["ttft_p50_ms"],
            "cores_busy": {"loadgen": round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / el, 2),
                           "mock": round((cpu_seconds(mock_proc.pid) - m0) / el, 2)},
            "what": "qmx_loadgen -> mock 0 directly (no proxy), same conns / threads / validation; a proxied "
                    "request of the scenario costs the mocks one stream per backend"}


def exit_status(p) -> dict:
    """How a harness process ended (None: still running)."""
    rc = p.poll()
    if rc is None:
        return {"pid": p.pid, "running": True}
    d = {"pid": p.pid, "running": False, "returncode": rc}
    if rc < 0:
        try:
            d["signal"] = signal.Signals(-rc).name
        except ValueError:
            d["signal"] = -rc
    return d


def spawn_reference(ref_root: str, tmp: str, cfg_path: str, port: int) -> subprocess.Popen:
    """The reference proxy, UNMODIFIED, from a scratch copy: quorum reads
    <copy>/config.yaml (oai_proxy.py:46) and writes <copy>/logs/ (oai_proxy.py:20-37); one
    uvicorn worker as in its Makefile (run-prod, Makefile:7).  Same mocks and load
    generator as the native proxy: the same-harness baseline BASELINE.md asks for."""
    import shutil

    copy = os.path.join(tmp, "refcopy")
    shutil.copytree(os.path.join(ref_root, "src"), os.path.join(copy, "src"))
    shutil.copy(cfg_path, os.path.join(copy, "config.yaml"))
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(copy, "src")
    env.setdefault("OPENAI_API_KEY", "bench")
    return subprocess.Popen([sys.executable, "-m", "uvicorn", "quorum.oai_proxy:app", "--host", "127.0.0.1",
                             "--port", str(port), "--workers", "1", "--log-level", "warning"],
                            cwd=copy, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True)


# labelled series bench.py reads (histogram buckets are skipped)
LABELED = ("qmx_syscalls_total", "qmx_spread_remote_ends_total", "qmx_upstream_failures_by_class_total")


def scrape(port):
    """Sum the proxy's /metrics counters (engine / kernel / tick / exchange) — one process
    per rank, io loops already aggregated inside it."""
    import urllib.request

    out = {}
    try:
        txt = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    except Exception:  # noqa: BLE001
        return out
    for ln in txt.splitlines():
        if not ln or ln[0] == "#" or ("{" in ln and not ln.startswith(LABELED)):
            continue
        k, _, v = ln.rpartition(" ")
        try:
            out[k] = float(v)
        except ValueError:
            pass
    return out


def cpu_seconds(pid: int) -> float:
    """utime + stime of a live process (all its threads), from /proc."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return 0.0


def rss_mb(pid: int) -> dict:
    """Resident memory of a live process (VmRSS) and its peak (VmHWM), MB, from /proc."""
    out = {}
    try:
        for ln in open(f"/proc/{pid}/status"):
            k, _, v = ln.partition(":")
            if k in ("VmRSS", "VmHWM"):
                out[k] = round(int(v.split()[0]) / 1024.0, 1)
    except (OSError, ValueError, IndexError):
        pass
    return out


def cgroup_cpu_stat() -> dict:
    """The job's cgroup CPU accounting (cgroup v2 cpu.stat + cpu.max): a CPU quota throttles
    every process of the job for the rest of a period once it is used up — latency spikes the
    breakdown should show, not hide."""
    out = {}
    for path, keys in (("/sys/fs/cgroup/cpu.stat", ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec")),):
        try:
            for ln in open(path):
                k, _, v = ln.partition(" ")
                if k in keys:
                    out[k] = int(v)
        except (OSError, ValueError):
            pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        out["quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return out


def cpu_snapshot(mock_procs, proxy_procs):
    import resource

    return {"proxy": sum(cpu_seconds(p.pid) for p in proxy_procs),
            "mocks": sum(cpu_seconds(p.pid) for p in mock_procs),
            "loadgen": resource.getrusage(resource.RUSAGE_CHILDREN).ru_utime
            + resource.getrusage(resource.RUSAGE_CHILDREN).ru_stime}


def cpu_breakdown(c0, c1, requests, elapsed):
    """CPU time per 1k completed requests by component (proxy / mock backends / load
    generator) over the timed region: the proxied-req/s metric shares the box's cores with
    the synthetic harness, so this says where the CPU goes."""
    d = {k: c1[k] - c0[k] for k in c0}
    out = {f"{k}_cpu_ms_per_1k_req": round(1e6 * v / max(requests, 1), 2) for k, v in d.items()}
    out["cores_busy"] = {k: round(v / elapsed, 2) for k, v in d.items()} if elapsed else {}
    return out


def breakdown(m0, m1, elapsed):
    d = {k: m1.get(k, 0.0) - m0.get(k, 0.0) for k in m1}
    launches = d.get("qmx_kernel_launches", 0.0)
    ticks = d.get("qmx_tick_seconds_count", 0.0)
    return {
        "ticks": int(ticks),
        "tick_wall_us_avg": round(1e6 * d.get("qmx_tick_seconds_sum", 0.0) / ticks, 1) if ticks else None,
        "streams_per_tick": round(d.get("qmx_tick_slots_total", 0.0) / ticks, 2) if ticks else None,
        "kernel_launches": int(launches),
        "tick_kernel_us_avg": round(1000 * d.get("qmx_kernel_kernel_ms", 0.0) / launches, 1) if launches else None,
        "tick_host_prep_us_avg": round(d.get("qmx_kernel_host_prep_us", 0.0) / launches, 1) if launches else None,
        "tick_launch_wait_us_avg": round(d.get("qmx_kernel_gpu_wait_us", 0.0) / launches, 1) if launches else None,
        "tick_process_us_avg": round(d.get("qmx_kernel_process_us", 0.0) / launches, 1) if launches else None,
        # posted -> first result record seen (doorbell / launch latency + the first item's run)
        "tick_first_result_us_avg": round(d.get("qmx_kernel_first_result_us", 0.0) / launches, 1) if launches else None,
        "tick_item_us_avg": round(d.get("qmx_kernel_item_us", 0.0) / launches, 1) if launches else None,
        "tick_start_spread_us_avg": round(d.get("qmx_kernel_start_spread_us", 0.0) / launches, 1) if launches else None,
        "tick_items_host_us_avg": round(d.get("qmx_kernel_items_host_us", 0.0) / launches, 1) if launches else None,
        # persistent grid, its own clock: doorbell seen -> relayed -> first item -> last item done
        "grid_us_avg": {k: round(d.get(f"qmx_kernel_{k}_us", 0.0) / d["qmx_kernel_grid_ticks"], 1)
                        for k in ("relay", "pickup", "grid_span")} if d.get("qmx_kernel_grid_ticks") else None,
        # loop ticks, host and device clocks calibrated against each other (HipGrid): the host's
        # post -> the relay saw it, the last item done -> the io loop took the results
        # (clock_window: the offset's remaining uncertainty, upper − lower bound per 100 ms window)
        "tick_hops_us_avg": dict({k: round(d.get(f"qmx_kernel_{k}_us", 0.0) / d["qmx_kernel_hop_ticks"], 1)
                                  for k in ("post_seen", "done_host")},
                                 clock_window=round(d["qmx_kernel_clock_window_us"] / d["qmx_kernel_clock_windows"], 2)
                                 if d.get("qmx_kernel_clock_windows") else None)
        if d.get("qmx_kernel_hop_ticks") else None,
        "tick_route_us_avg": round(1e6 * d.get("qmx_tick_route_seconds_total", 0.0) / ticks, 1) if ticks else None,
        # kernel seconds per wall second, SUMMED over the tick lanes (two lanes with kernels in
        # flight at once count twice): a lane-occupancy figure, not the GPU's busy fraction
        "kernel_s_per_s_lane_sum": round(d.get("qmx_kernel_kernel_ms", 0.0) / 1000 / elapsed, 4) if elapsed else None,
        # finalize (K3 strip + K4 join + K5 encode) rides the tick launches: requests folded into
        # them, and launches of its own (always 0 since r2)
        "finalize_items_fused": int(d.get("qmx_kernel_fin_items", 0.0)),
        "finalize_separate_launches": int(d.get("qmx_kernel_fin_separate_launches", 0.0)),
        "finalize_host": int(d.get("qmx_kernel_fin_host", 0.0)),
        "h2d_MB": round(d.get("qmx_kernel_h2d_bytes", 0.0) / 1e6, 2),
        "d2h_MB": round(d.get("qmx_kernel_d2h_bytes", 0.0) / 1e6, 2),
        "escalations": int(d.get("qmx_kernel_escalations", 0.0)),
        # streams opened on the host path by the latency mode (QMX_LIGHT_HOST)
        "light_host_opens": int(d.get("qmx_kernel_light_host_opens", 0.0)),
        # io-loop syscalls per request (sends to clients / upstreams, recvs, epoll, wakeups)
        "syscalls_per_req": {k.split('"')[1]: round(v / d["qmx_requests_total"], 2)
                             for k, v in d.items() if k.startswith("qmx_syscalls_total")}
        if d.get("qmx_requests_total") else {},
        "exchange_rounds": int(d.get("qmx_exchange_rounds_total", 0.0)),
        # deltas held for their stream's next output (more bytes already waiting) instead of a
        # client send of their own, per request
        "coalesced_per_req": (round(d.get("qmx_output_coalesced_total", 0.0) / d["qmx_requests_total"], 2)
                              if d.get("qmx_requests_total") else None),
        # the latency those holds added (hold start -> released) and the share the coalescing
        # deadline released rather than the stream's next output
        "hold_us_avg": (round(1e6 * d["qmx_output_hold_seconds_sum"] / d["qmx_output_hold_seconds_count"], 1)
                        if d.get("qmx_output_hold_seconds_count") else None),
        "hold_deadline_share": (round(d.get("qmx_output_hold_deadline_total", 0.0)
                                      / d["qmx_output_hold_seconds_count"], 3)
                                if d.get("qmx_output_hold_seconds_count") else None),
        # spread placement (EP): how the remote streams' finals moved — bulk rounds (RCCL
        # ncclSend/ncclRecv HBM -> HBM, or tcpbulk in rehearsals) vs the mesh — what the rounds
        # cost, and whether the owner finalized them on the GPU (HBM-resident / staged texts)
        "exchange": ({"remote_streams": int(d.get("qmx_remote_streams_total", 0.0)),
                      "bulk_rounds": int(d.get("qmx_exchange_rounds_total", 0.0)),
                      "round_us_avg": (round(d.get("qmx_exchange_busy_us_total", 0.0)
                                             / d["qmx_exchange_rounds_total"], 1)
                                       if d.get("qmx_exchange_rounds_total") else None),
                      "bulk_final_MB": round(d.get("qmx_exchange_bulk_bytes_total", 0.0) / 1e6, 3),
                      "eager_finals": int(d.get("qmx_spread_eager_finals_total", 0.0)),
                      "mesh_finals": int(d.get("qmx_exchange_mesh_finals_total", 0.0)),
                      "rescued": int(d.get("qmx_exchange_rescued_total", 0.0)),
                      "epochs": int(d.get("qmx_exchange_epochs_total", 0.0)),
                      "delta_mismatch": int(d.get("qmx_spread_delta_mismatch_total", 0.0)),
                      "worker_nodata": int(d.get("qmx_spread_worker_nodata_total", 0.0)),
                      "remote_texts_hbm": int(d.get("qmx_kernel_remote_texts_hbm", 0.0)),
                      "remote_texts_staged": int(d.get("qmx_kernel_remote_texts_staged", 0.0)),
                      "remote_texts_copied": int(d.get("qmx_kernel_remote_texts_copied", 0.0)),
                      # (RCCL at world > 1) copied HBM -> host by the exchange's bulk thread, and
                      # of them by an io loop instead (must stay 0: a device copy on the loop)
                      "host_copied_by_exchange": int(d.get("qmx_exchange_host_copied_total", 0.0)),
                      "copied_inline": int(d.get("qmx_kernel_remote_texts_copied_inline", 0.0)),
                      "release_deferred": int(d.get("qmx_spread_release_deferred_total", 0.0)),
                      "hops_us": hop_means(d)}
                     if d.get("qmx_remote_streams_total") else None),
        # where a request's time goes (server-side means over the timed region): upstream
        # TTFB (request sent -> first response bytes), engine wait (a stream's first bytes fed
        # -> its final result in the io loop: lane queueing + tick + routing), TTFT and whole
        # request as the proxy sees them
        "latency_us_avg": {k: round(1e6 * d[f"{m}_sum"] / d[f"{m}_count"], 1)
                           for k, m in (("upstream_ttfb", "qmx_upstream_ttfb_seconds"),
                                        ("engine_wait", "qmx_engine_wait_seconds"),
                                        ("tick", "qmx_tick_seconds"), ("ttft", "qmx_ttft_seconds"),
                                        ("request", "qmx_request_latency_seconds"))
                           if d.get(f"{m}_count")},
        # the io-loop / lane hand-offs around a tick (means): the oldest upstream bytes of an
        # io-loop iteration until they reach the engine, a dirty stream until a lane takes
        # it, a tick's results from routing until the io loop applies them
        "handoff_us_avg": {k: round(f * d[a] / d[b], 1)
                           for k, a, b, f in (("feed_to_engine", "qmx_flush_wait_seconds_total", "qmx_flushes_total", 1e6),
                                              ("dirty_to_taken", "qmx_engine_take_wait_us", "qmx_engine_takes", 1.0),
                                              ("routed_to_applied", "qmx_apply_wait_seconds_total", "qmx_applies_total", 1e6))
                           if d.get(b)},
        # QMX_STAGE_TIMING=1 runs only: in-kernel stage split per item (s_memrealtime stamps;
        # stages as tools/kbench.py) and the shader clock the items ran at
        "stage_us_per_item": ({k[11:]: round(v / d["qmx_kernel_stage_items"], 2)
                               for k, v in sorted(d.items())
                               if k.startswith("qmx_kernel_stage") and k.endswith("_us")}
                              if d.get("qmx_kernel_stage_items") else None),
        # ... and S3's event paths per item: full parses, stream-template and hole-template hits
        "s3_per_item": ({k[len("qmx_kernel_s3_"):]: round(d.get(k, 0.0) / d["qmx_kernel_stage_items"], 2)
                         for k in ("qmx_kernel_s3_events", "qmx_kernel_s3_full_parses", "qmx_kernel_s3_template_hits",
                                   "qmx_kernel_s3_hole_hits")}
                        if d.get("qmx_kernel_stage_items") else None),
        "shader_mhz": (round(d["qmx_kernel_clk_cycles"] / d["qmx_kernel_clk_us"], 1)
                       if d.get("qmx_kernel_clk_us") else None),
        # io-loop passes (epoll return -> next wait) over 1 / 5 ms in the timed region, and the
        # longest pass the process has had (not a delta): a blocked loop shows here
        # loop ticks: grid (re)launches and idle stops in the timed region, and the longest of
        # each the process had — every io loop that posts meanwhile waits for them
        "grid": ({"launches": int(d.get("qmx_kernel_grid_launches", 0.0)),
                  "stops": int(d.get("qmx_kernel_grid_stops", 0.0)),
                  "launch_ms_max": round(1e-3 * m1.get("qmx_kernel_grid_launch_us_max", 0.0), 2),
                  "calibrate_ms_max": round(1e-3 * m1.get("qmx_kernel_grid_launch_calibrate_us_max", 0.0), 2),
                  "stop_ms_max": round(1e-3 * m1.get("qmx_kernel_grid_stop_us_max", 0.0), 2)}
                 if "qmx_kernel_grid_launches" in m1 else None),
        "runtime_allocs": int(d.get("qmx_kernel_runtime_allocs", 0.0)),
        "runtime_alloc_ms": round(1e-3 * d.get("qmx_kernel_runtime_alloc_us", 0.0), 2),
        "loop_passes_over_1ms": int(d.get("qmx_loop_passes_over_1ms_total", 0.0)),
        "loop_passes_over_5ms": int(d.get("qmx_loop_passes_over_5ms_total", 0.0)),
        "loop_pass_max_ms": round(1e3 * m1.get("qmx_loop_pass_max_seconds", 0.0), 2),
        # HIP streams of the proxy process vs the hardware queues per priority level: a persistent
        # grid on an exclusive (highest-priority) stream has its queue to itself (qmx_streams.h)
        "hip_streams": ({"shared": int(m1.get("qmx_kernel_streams_shared", 0.0)),
                         "exclusive": int(m1.get("qmx_kernel_streams_exclusive", 0.0)),
                         "hw_queues_per_priority": int(m1.get("qmx_kernel_hw_queues_per_priority", 0.0)),
                         "grid_queue_exclusive": bool(m1.get("qmx_kernel_grid_queue_exclusive", 0.0)),
                         "grid_queue_ok": bool(m1.get("qmx_kernel_grid_queue_ok", 0.0))}
                        if "qmx_kernel_hw_queues_per_priority" in m1 else None),
    }


def compact_breakdown(rank: int, bd: dict, row) -> dict:
    """One rank's row of the JSON line: which process answered, its load and its key timings."""
    lat = bd.get("latency_us_avg", {})
    return {"rank": rank, "pid": bd.get("pid"), "requests": int(row[1]), "req_s": round(row[1] / row[0], 1) if row[0] else None,
            "p50_ttft_ms": round(row[2], 3), "ticks": bd.get("ticks"), "streams_per_tick": bd.get("streams_per_tick"),
            "tick_kernel_us_avg": bd.get("tick_kernel_us_avg"), "tick_wall_us_avg": bd.get("tick_wall_us_avg"),
            "engine_wait_us": lat.get("engine_wait"), "proxy_cpu_ms_per_1k_req": bd.get("proxy_cpu_ms_per_1k_req"),
            "finalize_host": bd.get("finalize_host"), "exchange": bd.get("exchange")}


def spread_summary(rows) -> dict:
    """The spread check of every rank, compact: totals plus each rank's own counters.  ``main``:
    the production defaults under load (short final texts eager); ``rendezvous``: every final
    text through a bulk round (RCCL on GPUs, tcpbulk in rehearsals); ``local``: the control."""
    def med(vals):
        vals = [v for v in vals if v is not None]
        return round(statistics.median(vals), 3) if vals else None

    def get(r, *path):
        for k in path:
            r = (r or {}).get(k)
        return r

    def tot(*path):
        return int(sum(get(r, *path) or 0 for r in rows))

    def ends(*path):
        e = {}
        for r in rows:
            for k, v in (get(r, *path) or {}).items():
                e[k] = e.get(k, 0) + int(v)
        return e

    def hops(*path):
        hs = [get(r, *path) or {} for r in rows]
        return {k: med([h.get(k) for h in hs]) for k in ("open_to_first_delta", "last_delta_to_final")}

    passes = [("main", "load"), ("main", "probe"), ("rendezvous", "load"), ("rendezvous", "probe"), ("local", "probe")]
    out = {"ok": all(r.get("ok") for r in rows), "transport": rows[0].get("transport"),
           # main set under load (32 connections per rank, 2048 requests each)
           "requests": tot("main", "load", "requests"),
           "invalid": sum(tot(a, b, "invalid") for a, b in passes),
           "remote_streams": tot("main", "load", "remote_streams"),
           "eager_finals": tot("main", "load", "eager_finals"),
           "mesh_finals": tot("main", "load", "mesh_finals") + tot("rendezvous", "load", "mesh_finals"),
           "delta_mismatch": sum(tot(a, b, "delta_mismatch") for a, b in passes[:4]),
           "worker_nodata": sum(tot(a, b, "worker_nodata") for a, b in passes[:4]),
           "peer_downs": sum(tot(a, b, "peer_downs") for a, b in passes[:4]),
           # merged sessions finalized on the owner's host instead of its GPU (0 expected)
           "finalize_host": sum(tot(a, b, "finalize_host") for a, b in passes[:4]),
           "remote_texts_gpu": {"hbm": sum(tot(a, b, "remote_texts_hbm") for a, b in passes[:4]),
                                "staged": sum(tot(a, b, "remote_texts_staged") for a, b in passes[:4]),
                                "copied": sum(tot(a, b, "remote_texts_copied") for a, b in passes[:4])},
           "remote_ends": ends("main", "load", "remote_ends"),
           "p50_latency_ms": med([get(r, "main", "load", "p50_latency_ms") for r in rows]),
           "hops_us_loaded": hops("main", "load", "hops_us"),
           # one session at a time per rank: spread (defaults) vs the same config placed locally
           "probe_p50_latency_ms": med([get(r, "main", "probe", "p50_latency_ms") for r in rows]),
           "local_probe_p50_latency_ms": med([get(r, "local", "probe", "p50_latency_ms") for r in rows]),
           "hops_us_probe": hops("main", "probe", "hops_us"),
           # every final text through a round: the RCCL / tcpbulk round protocol exercised
           "bulk_formed": all(get(r, "rendezvous", "bulk_formed") for r in rows),
           "bulk_rounds": tot("rendezvous", "load", "bulk_rounds") + tot("rendezvous", "probe", "bulk_rounds"),
           "rendezvous": {"requests": tot("rendezvous", "load", "requests") + tot("rendezvous", "probe", "requests"),
                          "bulk_final_bytes": tot("rendezvous", "load", "bulk_final_bytes")
                          + tot("rendezvous", "probe", "bulk_final_bytes"),
                          "remote_ends": ends("rendezvous", "load", "remote_ends"),
                          "p50_latency_ms": med([get(r, "rendezvous", "load", "p50_latency_ms") for r in rows]),
                          "probe_p50_latency_ms": med([get(r, "rendezvous", "probe", "p50_latency_ms") for r in rows]),
                          "hops_us_probe": hops("rendezvous", "probe", "hops_us")}}
    degraded = [f"rank {i}: {get(r, 'rendezvous', 'degraded')}" for i, r in enumerate(rows)
                if get(r, "rendezvous", "degraded")]
    if degraded:  # the round protocol did not run somewhere (finals took the mesh, validated)
        out["degraded"] = degraded[:8]
    errs = [f"rank {i} {k}: {get(r, k, 'error')}" for i, r in enumerate(rows) for k in ("main", "rendezvous", "local")
            if get(r, k, "error")]
    if errs or any(r.get("error") for r in rows):
        out["errors"] = (errs + [f"rank {i}: {r['error']}" for i, r in enumerate(rows) if r.get("error")])[:8]

    def compact(d):
        keep = ("requests", "invalid", "p50_latency_ms", "remote_streams", "eager_finals", "bulk_rounds", "mesh_finals",
                "delta_mismatch", "worker_nodata", "remote_ends", "up_failures", "hops_us", "finalize_host",
                "remote_texts_hbm", "remote_texts_staged", "remote_texts_copied", "error")
        return {k: v for k, v in (d or {}).items() if k in keep and v}

    def rank_error(r):
        e = [f"{k}: {get(r, k, 'error')}" for k in ("main", "rendezvous", "local") if get(r, k, "error")]
        return "; ".join(e + ([r["error"]] if r.get("error") else [])) or None

    out["per_rank"] = [{"ok": r.get("ok"), "pid": get(r, "main", "pid"), "error": rank_error(r),
                        **{f"{a}_{b}": compact(get(r, a, b)) for a, b in passes}} for r in rows]
    return out


def spread_check(args, sc, rank, world, engine, device, bin_dir, tmp, mock_ports, dist, n_dev):
    """Outside the timed region, N > 1: expert-parallel placement end to end, on three proxy
    sets of the headline backends with the final event on (skip_final_aggregation: false), so
    backend 1 of every session runs on the next rank and its deltas cross the TCP mesh:

    * ``main`` (port + 50): the production defaults under load — a final text up to
      ``exchange_eager_bytes`` rides the mesh behind its deltas (eager), a longer one takes a
      bulk round — then a one-connection latency probe;
    * ``rendezvous`` (port + 20): every final text through a bulk round (rank 0 numbers the
      rounds; RCCL ncclSend/ncclRecv HBM → HBM on GPUs, the socket executor in rehearsals),
      a lighter load and the probe;
    * ``local`` (port + 80): the same config placed locally — the probe's control.

    Every response is validated; the exchange counters say which path moved the finals.
    Failures are reported, never hidden (``checks_ok: false`` and a warning), and do not
    touch the headline measurement, whose validity covers the timed region."""
    from quorum_amd.parallel.exchange import exchange_env

    on_gpu = n_dev >= world
    spec = os.path.join(tmp, "expect_spread.txt")
    prep_err = None
    try:
        expect_spec(spec, sc, False, mock_expected(bin_dir))
    except Exception as e:  # noqa: BLE001
        prep_err = repr(e)[:300]
    if not torch_min_flag(dist, prep_err is None, on_gpu):
        return {"ok": False, "error": prep_err or "another rank failed to prepare the spread check"}
    # ranks sharing a GPU (rehearsal) or no GPU: RCCL needs one GPU per rank, so the same
    # bulk rounds run with the socket executor (tcpbulk)
    xchg = os.environ.get("QMX_XCHG") or ("rccl" if on_gpu and engine == "hip" else "tcpbulk")
    if xchg == "rccl" and not (on_gpu and engine == "hip"):
        xchg = "tcpbulk"

    def xenv(off, **extra):
        nonce = [str(time.time_ns()) if rank == 0 else None]
        dist.broadcast_object_list(nonce, src=0)
        # a bulk round that cannot complete (a communicator that formed but does not move
        # bytes) gives up after 3 s, not the production 30 s: its texts fall back to the mesh
        # and the check still validates every response inside the load generator's window
        e = dict(exchange_env(rank, world, args.port + off, nonce[0]), QMX_XCHG=xchg,
                 QMX_XCHG_TIMEOUT=os.environ.get("QMX_XCHG_TIMEOUT", "3"))
        e.update(extra)
        return e

    ctx = {"args": args, "rank": rank, "dist": dist, "on_gpu": on_gpu, "tmp": tmp, "mock_ports": mock_ports, "sc": sc,
           "engine": engine, "device": device, "bin_dir": bin_dir, "spec": spec}
    main = run_set(ctx, "spread", "spread", args.port + 50, args.port + SPREAD_ADMIN_OFF + rank, xenv(50),
                   [("load", 32, 2048), ("probe", 1, PROBE_REQUESTS)])
    rdv = run_set(ctx, "spread_rendezvous", "spread", args.port + 20, args.port + RDV_ADMIN_OFF + rank,
                  xenv(20, QMX_XCHG_EAGER_BYTES="0"), [("load", 8, 512), ("probe", 1, PROBE_REQUESTS)], want_bulk=True)
    local = run_set(ctx, "spread_local", "local", args.port + 80, args.port + LOCAL_ADMIN_OFF + rank, {},
                    [("probe", 1, PROBE_REQUESTS)])
    return {"ok": main["ok"] and rdv["ok"] and local["ok"], "transport": xchg, "main": main, "rendezvous": rdv,
            "local": local}


def config3_check(args, rank, world, engine, device, bin_dir, tmp, mock_ports, dist, n_dev):
    """Outside the headline's timed region, N > 1: BASELINE config 3 measured — 4 mock
    backends, streaming aggregate strategy, sessions sharded over the ranks AND each
    session's backend streams spread over them (backend i on rank owner + i), with EVERY
    remote final text moved by a bulk round (exchange_eager_bytes 0): RCCL ncclSend /
    ncclRecv HBM -> HBM on a GPU node (tcpbulk when ranks share a GPU), then the owner's
    fused GPU finalize (K3 / K4 texts for the aggregator prompt).  One timed, validated pass
    per rank; its req/s, TTFT, round counts and costs are reported under ``config3``."""
    from quorum_amd.parallel.exchange import exchange_env

    sc = SCENARIOS["aggregate4"]
    on_gpu = n_dev >= world
    xchg = os.environ.get("QMX_XCHG") or ("rccl" if on_gpu and engine == "hip" else "tcpbulk")
    if xchg == "rccl" and not (on_gpu and engine == "hip"):
        xchg = "tcpbulk"
    extra, prep_err = [], None
    ports = list(mock_ports)
    try:
        for i in range(len(ports), sc["n"]):  # the headline ran 2 backends: 2 more mocks
            p = args.port + 100 + rank * 10 + i
            extra.append(subprocess.Popen([os.path.join(bin_dir, "qmx_mock"), "--port", str(p), "--threads",
                                           str(args.mock_threads), "--tokens", "20", "--think", "1"],
                                          stderr=subprocess.DEVNULL, start_new_session=True))
            ports.append(p)
        spec = os.path.join(tmp, "expect_config3.txt")
        expect_spec(spec, sc, False, mock_expected(bin_dir))
    except Exception as e:  # noqa: BLE001
        prep_err = repr(e)[:300]
    try:
        if not torch_min_flag(dist, prep_err is None, on_gpu):
            return {"ok": False, "error": prep_err or "another rank failed to prepare the config-3 pass"}
        nonce = [str(time.time_ns()) if rank == 0 else None]
        dist.broadcast_object_list(nonce, src=0)
        xenv = dict(exchange_env(rank, world, args.port + 60, nonce[0]), QMX_XCHG=xchg, QMX_XCHG_EAGER_BYTES="0",
                    QMX_XCHG_TIMEOUT=os.environ.get("QMX_XCHG_TIMEOUT", "3"))
        ctx = {"args": args, "rank": rank, "dist": dist, "on_gpu": on_gpu, "tmp": tmp, "mock_ports": ports, "sc": sc,
               "engine": engine, "device": device, "bin_dir": bin_dir, "spec": spec}
        res = run_set(ctx, "config3", "spread", args.port + 60, args.port + C3_ADMIN_OFF + rank, xenv,
                      [("load", 16, CONFIG3_REQUESTS)], want_bulk=True)
        res["transport"] = xchg
        return res
    finally:
        _kill(extra)


def config3_summary(rows) -> dict:
    """The config-3 pass of every rank: node req/s (total requests / slowest rank's wall),
    validation, and how the remote finals moved (rounds, their mean duration, bytes)."""
    loads = [(r or {}).get("load") or {} for r in rows]
    walls = [l["requests"] / l["req_s"] for l in loads if l.get("req_s")]
    reqs = sum(int(l.get("requests", 0)) for l in loads)
    out = {"ok": all((r or {}).get("ok") for r in rows), "transport": (rows[0] or {}).get("transport"),
           "scenario": "aggregate4 + placement spread, exchange_eager_bytes 0 (every remote final through a round)",
           "requests": reqs, "req_s": round(reqs / max(walls), 1) if walls else None,
           "p50_ttft_ms": (round(statistics.median(l["p50_ttft_ms"] for l in loads if l.get("p50_ttft_ms") is not None), 3)
                           if any(l.get("p50_ttft_ms") is not None for l in loads) else None),
           "invalid": sum(int(l.get("invalid", 0)) for l in loads),
           "bulk_rounds": int(sum(l.get("bulk_rounds", 0) for l in loads)),
           "bulk_final_MB": round(sum(l.get("bulk_final_bytes", 0) for l in loads) / 1e6, 3),
           "mesh_finals": int(sum(l.get("mesh_finals", 0) for l in loads)),
           "finalize_host": int(sum(l.get("finalize_host", 0) for l in loads)),
           "remote_texts_gpu": {"hbm": int(sum(l.get("remote_texts_hbm", 0) for l in loads)),
                                "staged": int(sum(l.get("remote_texts_staged", 0) for l in loads)),
                                "copied": int(sum(l.get("remote_texts_copied", 0) for l in loads))},
           "delta_mismatch": int(sum(l.get("delta_mismatch", 0) for l in loads)),
           "per_rank": [{"requests": l.get("requests"), "req_s": l.get("req_s"), "bulk_rounds": l.get("bulk_rounds"),
                         "round_us_avg": l.get("round_us_avg"), "hops_us": l.get("hops_us")} for l in loads]}
    errs = [f"rank {i}: {(r or {}).get('error')}" for i, r in enumerate(rows) if (r or {}).get("error")]
    if errs:
        out["errors"] = errs[:8]
    deg = [f"rank {i}: {(r or {}).get('degraded')}" for i, r in enumerate(rows) if (r or {}).get("degraded")]
    if deg:
        out["degraded"] = deg[:8]
    return out


def spread_counters(d) -> dict:
    """A spread proxy's /metrics delta over one pass: how its remote streams moved and ended."""
    return {"remote_streams": d.get("qmx_remote_streams_total", 0.0),
            "eager_finals": d.get("qmx_spread_eager_finals_total", 0.0),
            "bulk_rounds": d.get("qmx_exchange_rounds_total", 0.0),
            "bulk_final_bytes": d.get("qmx_exchange_bulk_bytes_total", 0.0),
            "round_us_avg": (round(d.get("qmx_exchange_busy_us_total", 0.0) / d["qmx_exchange_rounds_total"], 1)
                             if d.get("qmx_exchange_rounds_total") else None),
            "mesh_finals": d.get("qmx_exchange_mesh_finals_total", 0.0),
            "mesh_messages": d.get("qmx_exchange_messages_total", 0.0),
            "delta_mismatch": d.get("qmx_spread_delta_mismatch_total", 0.0),
            "worker_nodata": d.get("qmx_spread_worker_nodata_total", 0.0),
            "peer_downs": d.get("qmx_exchange_peer_downs_total", 0.0),
            # the owner's finalize of merged sessions: on the host (should stay 0: remote texts
            # sit in HBM after an RCCL round, or are staged into the GPU finalize items)
            "finalize_host": d.get("qmx_kernel_fin_host", 0.0),
            "remote_texts_hbm": d.get("qmx_kernel_remote_texts_hbm", 0.0),
            "remote_texts_staged": d.get("qmx_kernel_remote_texts_staged", 0.0),
            "remote_texts_copied": d.get("qmx_kernel_remote_texts_copied", 0.0),
            # how this rank's remote streams ended (owner side), and its upstream failures by
            # class (worker side included)
            "remote_ends": {k.split('"')[1]: v for k, v in d.items() if k.startswith("qmx_spread_remote_ends_total") and v},
            "up_failures": {k.split('"')[1]: v for k, v in d.items()
                            if k.startswith("qmx_upstream_failures_by_class_total") and v},
            # owner side, means: X_OPEN -> first delta back; last delta -> final applied
            "hops_us": hop_means(d)}


def run_set(ctx, label, placement, port, admin, xenv, passes, want_bulk=False) -> dict:
    """One proxy per rank on ``port`` (``placement``; ``xenv``: its exchange settings): wait
    until every rank's is up (spread: its mesh formed; ``want_bulk``: its bulk executor too, at
    most 60 s), run each pass ``(name, connections, requests)`` of validated requests, and stop
    the set.  Every rank joins the same collectives whatever fails locally: a rank's counters
    are read only after every rank's pass is done (a spread rank serves its peers' remote
    streams to the end).  The result, or the failure, as a dict."""
    from quorum_amd.serve import spawn_workers, wait_healthy

    args, rank, dist, on_gpu = ctx["args"], ctx["rank"], ctx["dist"], ctx["on_gpu"]
    res, procs, err = {}, [], None
    try:
        if label == "spread" and os.environ.get("QMX_BENCH_SPREAD_FAIL_RANK") == str(rank):  # test hook
            raise RuntimeError("injected spread-check failure")
        cfg = os.path.join(ctx["tmp"], f"config_{label}.yaml")
        write_config(cfg, ctx["mock_ports"], False, args.tile, ctx["sc"], placement)
        env = dict(os.environ, **xenv, QMX_READY_FILE=os.path.join(ctx["tmp"], f"ready_{label}"),
                   QMX_ADMIN_PORT=str(admin))
        procs = spawn_workers(cfg, "127.0.0.1", port, 1, ctx["engine"], ctx["device"], impl="native",
                              threads=args.threads, env=env)
        for p in procs:
            p.ready_file = f"{env['QMX_READY_FILE']}.{p.pid}"
        res["pid"] = procs[0].pid if procs else None
        if not (wait_ready(procs, 60) and wait_healthy("127.0.0.1", admin, 30)):
            raise RuntimeError(f"{label} proxy did not become ready: {[exit_status(p) for p in procs]}")
    except Exception as e:  # noqa: BLE001
        err = repr(e)[:300]
    up = torch_min_flag(dist, err is None, on_gpu)
    if up and placement == "spread":
        try:
            t0, bulk = time.time(), False
            while True:  # the mesh formed on every rank (and the bulk executor: RCCL communicator)
                m = scrape(admin)
                healthy = m.get("qmx_exchange_healthy") == 1.0
                bulk = m.get("qmx_exchange_rccl_active") == 1.0
                if healthy and (not want_bulk or bulk):
                    break
                if time.time() - t0 > 60:
                    if not healthy:
                        raise RuntimeError(f"{label}: exchange did not form: "
                                           f"{({k: v for k, v in m.items() if 'exchange' in k})}")
                    # no communicator: the finals fall back to the mesh (still validated);
                    # reported, so a node where RCCL never formed is visible in the line
                    break
                time.sleep(0.2)
            res["bulk_formed"] = bulk
        except Exception as e:  # noqa: BLE001
            err = repr(e)[:300]
        up = torch_min_flag(dist, err is None, on_gpu)
    for name, conns, n in passes:
        if not up:
            break
        # a pass's counters are this rank's deltas, but its sessions shard over every rank's
        # proxy (SO_REUSEPORT) and their streams spread over the ranks: every rank takes its
        # baseline before any rank's load starts, and its final scrape before any rank's
        # next pass does (a fast rank's probe would otherwise land in a slow rank's load)
        st, m0 = None, scrape(admin)
        torch_min_flag(dist, True, on_gpu)
        try:
            st = loadgen(ctx["bin_dir"], port, conns, n, min(2, conns), 120, ctx["spec"])
        except Exception as e:  # noqa: BLE001
            err = repr(e)[:300]
        up = torch_min_flag(dist, err is None, on_gpu)  # every rank's pass is done
        time.sleep(0.1)
        m1 = scrape(admin)
        torch_min_flag(dist, True, on_gpu)
        if st is not None:
            d = {k: v - m0.get(k, 0.0) for k, v in m1.items()}
            res[name] = {"ok": st["invalid"] == 0 and st["errors"] == 0 and st["completed"] == n,
                         "requests": st["completed"], "invalid": st["invalid"], "errors": st["errors"],
                         "p50_latency_ms": st["lat_p50_ms"], "p50_ttft_ms": st["ttft_p50_ms"], "req_s": st["rps"]}
            if placement == "spread":
                res[name].update(spread_counters(d))
                # validated bytes are not enough: a delta-count mismatch or a worker stream that
                # sent nothing for its content breaks the spread invariants
                if res[name]["delta_mismatch"] or res[name]["worker_nodata"]:
                    res[name]["ok"] = False
    _kill(procs)
    if err is None and not up:
        err = f"another rank's {label} set failed"
    if err is None and want_bulk:
        # the rendezvous set exists to run the round protocol: no communicator, or no round on
        # this rank, is reported as DEGRADED (its finals fell back to the mesh and were still
        # validated), never as a silent pass — and never hidden inside "ok"
        rounds = sum((res.get(p[0]) or {}).get("bulk_rounds", 0) for p in passes)
        if not res.get("bulk_formed") or rounds <= 0:
            res["degraded"] = f"{label}: bulk rounds did not run (formed {res.get('bulk_formed')}, rounds {rounds})"
    res["ok"] = err is None and all((res.get(p[0]) or {}).get("ok") for p in passes)
    if err:
        res["error"] = err
    return res


def torch_min_flag(dist, flag: bool, on_gpu: bool) -> bool:
    """min over ranks of a bool (an all-reduce every rank joins)."""
    import torch

    t = torch.tensor([1.0 if flag else 0.0], device="cuda" if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return t.item() >= 1.0


def hop_means(d) -> dict:
    """Spread hop means (µs) from a /metrics delta: X_OPEN -> first delta, last delta -> final."""
    return {k: round(1e6 * d[f"{m}_sum"] / d[f"{m}_count"], 1)
            for k, m in (("open_to_first_delta", "qmx_spread_first_delta_seconds"),
                         ("last_delta_to_final", "qmx_spread_final_seconds"))
            if d.get(f"{m}_count")}


def self_launch(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start ``torch.distributed.run
    --nproc-per-node N`` on this same command line as a CHILD process (never an exec: nothing
    here has touched the GPU, and the ranks must own their devices), relay its output and
    exit with its code.  The driver's own torchrun invocation sets WORLD_SIZE and skips this."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        mport = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", str(mport)),
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: --gpus {n}: launching {n} ranks: {' '.join(cmd[1:7])} ...", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd)

    def fwd(signum, _frame):
        try:
            p.send_signal(signum)
        except OSError:
            pass

    old = {sg: signal.signal(sg, fwd) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        return p.wait()
    finally:
        for sg, h in old.items():
            signal.signal(sg, h)


def wait_ready(procs, timeout: float) -> bool:
    """Every proxy process of THIS rank has written its ready file (``QMX_READY_FILE`` +
    ``.pid``, written once all its io loops listen): readiness of this rank's own workers,
    not of whichever rank's proxy answers on the shared SO_REUSEPORT port."""
    t0 = time.time()
    while time.time() - t0 < timeout:
        if any(p.poll() is not None for p in procs):
            return False
        if all(os.path.exists(p.ready_file) for p in procs):
            return True
        time.sleep(0.05)
    return False


def main() -> int:
    # the bench measures the GPU path itself: serve's latency mode (idle loops' streams on the
    # HIP engine's host path) stays off unless asked for (QMX_LIGHT_HOST=N)
    os.environ.setdefault("QMX_LIGHT_HOST", "0")
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without WORLD_SIZE: launches them (torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0,
                    help="requests per step per rank (0: the scenario's default, 131072 headline / 4096 others)")
    ap.add_argument("--conns", type=int, default=64, help="concurrent client connections per rank")
    ap.add_argument("--impl", default=os.environ.get("QMX_BENCH_IMPL", "native"),
                    choices=["native", "python", "reference"],
                    help="reference: the unmodified upstream proxy (scratch copy of --ref-root) under uvicorn, "
                         "same mocks and load generator (same-harness baseline)")
    ap.add_argument("--ref-root", default=os.environ.get("QMX_REF_ROOT") or next(
        (d for d in ("/root/reference", os.path.join(ROOT, ".refstage")) if os.path.isdir(os.path.join(d, "src"))),
        "/root/reference"),
        help="reference checkout (its src/ is copied to a scratch dir); .refstage/ is a git-ignored staging "
             "copy for GPU boxes, which have no /root/reference")
    ap.add_argument("--engine", default=os.environ.get("QMX_BENCH_ENGINE", "auto"))
    ap.add_argument("--workers", type=int, default=4, help="python impl: proxy processes per rank")
    ap.add_argument("--threads", type=int, default=0,
                    help="native impl: io threads per rank (0: min(8, cores / (2 x ranks)), at least 2 — "
                         "the node's cores are shared by every rank's proxy, mocks and load generator)")
    # load-generator threads (every response is validated; the envelope fast path costs ~2-5
    # us per response): 0 = 4 when the bench is bound to a compact CPU set (408-425k req/s vs
    # 372-374k with 3, p50 TTFT 0.12 vs 0.15 ms), else 3 (unbound, a 4th thread measured
    # slower: 261k vs 301k) — profiles/r5/pinning
    ap.add_argument("--lg-threads", type=int, default=0)
    ap.add_argument("--mock-threads", type=int, default=2)
    ap.add_argument("--skip-final", type=int, default=1)
    ap.add_argument("--tile", type=int, default=16384)
    ap.add_argument("--port", type=int, default=int(os.environ.get("QMX_BENCH_PORT", "18000")))
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--scenario", default="headline", choices=sorted(SCENARIOS))
    ap.add_argument("--spread-check", type=int, default=1,
                    help="N > 1: after the timed steps, validate spread placement (RCCL finals) end to end")
    ap.add_argument("--placement", default="local", choices=["local", "spread"],
                    help="spread: a session's backend streams run on consecutive ranks (RCCL exchange)")
    ap.add_argument("--ceiling", type=float, default=2.0,
                    help="seconds of the harness-ceiling check after the timed region (the load generator straight "
                         "against one mock, no proxy: harness_ceiling_req_s); 0 skips it")
    ap.add_argument("--plan", action="store_true",
                    help="print the per-rank thread / CPU plan for --gpus N on this node (QMX_SYSFS_ROOT: a "
                         "copy of /sys; QMX_BENCH_QUOTA: the CPU quota) and exit — nothing is launched or bound")
    ap.add_argument("--eager-bytes", type=int, default=-1,
                    help="spread: final texts up to this size ride the mesh behind their deltas (-1: the "
                         "production default, 4 KiB); 0 sends every remote final text through a bulk round "
                         "(RCCL ncclSend/ncclRecv HBM -> HBM on GPUs; tcpbulk when ranks share a GPU)")
    args = ap.parse_args()
    if args.plan:
        from quorum_amd.parallel.topology import all_node_cpus, gpu_numa_nodes

        world = args.gpus or 1
        quota = int(os.environ.get("QMX_BENCH_QUOTA") or available_cores())
        allowed = (all_node_cpus() if os.environ.get("QMX_SYSFS_ROOT") else sorted(os.sched_getaffinity(0)))
        nodes = gpu_numa_nodes()
        nodes = [max(0, nodes[r % len(nodes)]) if nodes else 0 for r in range(world)]
        print(json.dumps(node_plan(world, SCENARIOS[args.scenario], args, quota, allowed, nodes)), flush=True)
        return 0
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is not None and args.gpus > 1 and env_world is None:
        return self_launch(args.gpus)
    if args.gpus is not None and env_world is not None and int(env_world) != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to measure a different "
              f"world than the one requested", file=sys.stderr, flush=True)
        return 2
    sc = SCENARIOS[args.scenario]
    if "conns" in sc and args.conns == 64:  # scenario default unless set explicitly
        args.conns = sc["conns"]
    if args.impl == "reference" and args.conns == 64:
        args.conns = 16  # the survey's reference rows (16 clients)
    if args.batch <= 0:
        # the reference serves ~9 req/s: 64 requests per step keeps a default run in minutes
        args.batch = 64 if args.impl == "reference" else sc.get("batch", 4096)
    skip_final = bool(args.skip_final) if args.scenario == "headline" else sc["skip"]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.threads <= 0:
        args.threads = max(2, min(8, available_cores() // (2 * world)))

    _trace_watch()
    import torch

    _trace("import torch")
    # QMX_BENCH_NDEV: a rehearsal names the GPU count itself, so the bench processes never
    # open the device (a box counts every process holding it open)
    n_dev = int(os.environ["QMX_BENCH_NDEV"]) if os.environ.get("QMX_BENCH_NDEV") else torch.cuda.device_count()
    # one rank per GPU (the driver's node runs); a rehearsal with more ranks than GPUs maps
    # ranks onto the visible GPUs, keeps the bench's own bookkeeping group on gloo (RCCL
    # refuses two ranks on one GPU) and keeps the bench processes themselves off the GPU:
    # they do no GPU work (the native workers do), and a box admits 16 GPU processes
    use_cuda = n_dev >= world and n_dev > 0 and torch.cuda.is_available()
    _trace("device count")
    device = local_rank % n_dev if n_dev else None
    coll_cuda = use_cuda
    dist = None
    if use_cuda:  # before the process group: RCCL's barrier picks the current device
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("nccl" if coll_cuda else "gloo")
    _trace("init_process_group")
    try:
        pinning = pin_rank(torch, world, local_rank, n_dev)
        if pinning is None and world == 1:
            pinning = pin_single(torch, n_dev)
    except (OSError, RuntimeError, ValueError, AttributeError) as e:  # placement is an optimisation only
        pinning = {"pinned": False, "error": repr(e)}
    if args.lg_threads <= 0:
        args.lg_threads = 4 if (pinning or {}).get("pinned") else 3
    engine = args.engine
    if engine == "auto":  # BASELINE config 1 is the CPU plumbing path; the rest run on the GPU
        engine = sc.get("engine") or ("hip" if n_dev else "cpu")
    direct = bool(sc.get("direct"))
    stream = bool(sc.get("stream", True))

    from quorum_amd.ops import build as qbuild

    qbuild.build()
    bin_dir = os.path.dirname(str(qbuild.build_tools()[0]))
    from quorum_amd.parallel.exchange import exchange_env
    from quorum_amd.parallel.topology import summary as link_summary
    from quorum_amd.serve import spawn_workers, wait_healthy

    procs = []
    tmp = tempfile.mkdtemp(prefix=f"qmx_bench_r{rank}_")
    ok = True
    try:
        mock_ports = [args.port + 100 + rank * 10 + i for i in range(sc["n"])]
        for i, p in enumerate(mock_ports):
            procs.append(subprocess.Popen([os.path.join(bin_dir, "qmx_mock"), "--port", str(p), "--threads",
                                           str(args.mock_threads), "--tokens", "20", "--think", "1"]
                                          + sc.get("mock_args", []) + sc["faults"].get(i, []),
                                          stderr=subprocess.DEVNULL, start_new_session=True))
        cfg_path = os.path.join(tmp, "config.yaml")
        write_config(cfg_path, mock_ports, skip_final, args.tile, sc, args.placement)
        spec_path = os.path.join(tmp, "expect.txt")
        expect_spec(spec_path, sc, skip_final, mock_expected(bin_dir))
        env = dict(os.environ)
        if n_dev:  # processes sharing this rank's GPU (persistent tick grids need it alone)
            env["QMX_GPU_SHARERS"] = str(max(1, -(-int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) // n_dev)))
        xchg_kind = None
        # QMX_SPREAD_SELF=1 at one rank (GPU rehearsal of the multi-rank path): the odd backends
        # of every session go through the rank's own exchange, final texts in RCCL rounds to itself
        self_spread = args.placement == "spread" and world == 1 and os.environ.get("QMX_SPREAD_SELF") == "1"
        if args.placement == "spread" and (world > 1 or self_spread):
            nonce = [str(time.time_ns()) if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(nonce, src=0)
            env.update(exchange_env(rank, world, args.port, nonce[0]))
            # RCCL needs one GPU per rank: ranks sharing a GPU (a rehearsal) run the same bulk
            # rounds with the socket executor
            xchg_kind = os.environ.get("QMX_XCHG") or ("rccl" if n_dev >= world and engine == "hip" else "tcpbulk")
            if xchg_kind == "rccl" and not (n_dev >= world and engine == "hip"):
                xchg_kind = "tcpbulk"
            env["QMX_XCHG"] = xchg_kind
            if args.eager_bytes >= 0:
                env["QMX_XCHG_EAGER_BYTES"] = str(args.eager_bytes)
        mock_procs = list(procs)
        proxy_port = args.port
        # this rank's own proxy process answers on admin_port (no SO_REUSEPORT): its ready
        # file says when it listens, and /metrics is scraped there — never through the shared
        # port, where any rank's proxy may answer
        admin_port = args.port + ADMIN_OFF + rank
        if direct:  # no proxy: the load generator talks to the mock itself
            proxy_port = mock_ports[0]
            proxy_procs = []
        elif args.impl == "reference":
            proxy_port = args.port + rank  # uvicorn binds without SO_REUSEPORT: a port per rank
            proxy_procs = [spawn_reference(args.ref_root, tmp, cfg_path, proxy_port)]
            admin_port = proxy_port
        else:
            env["QMX_READY_FILE"] = os.path.join(tmp, "ready")
            env["QMX_ADMIN_PORT"] = str(admin_port)
            if world > 1 and os.environ.get("QMX_BENCH_RANK_PORTS", "1") != "0":
                # client-side sharding: this rank's load generator drives this rank's proxy
                # only (its own port), not every rank's through the shared SO_REUSEPORT port —
                # the same per-rank share of sessions, without the co-located client's loopback
                # crossing L3s and sockets to the other ranks' proxies.  Rehearsal on one GPU,
                # ranks bound to L3s (QMX_BENCH_PIN_REHEARSE): 229k -> 318k req/s at 2 ranks,
                # 464k -> 589k at 4 (profiles/r5/rankports); QMX_BENCH_RANK_PORTS=0: shared port
                proxy_port = args.port + RANK_PORT_OFF + rank
            proxy_procs = spawn_workers(cfg_path, "127.0.0.1", proxy_port, args.workers, engine,
                                        device, impl=args.impl, threads=args.threads, env=env)
            for p in proxy_procs:
                p.ready_file = f"{env['QMX_READY_FILE']}.{p.pid}"
        procs += proxy_procs
        _trace("workers spawned")
        if direct:
            up = wait_port("127.0.0.1", proxy_port, 30)
        elif args.impl == "reference":
            up = wait_healthy("127.0.0.1", proxy_port, 180)
        else:
            up = wait_ready(proxy_procs, 180)
            if up and args.impl == "native":
                up = wait_healthy("127.0.0.1", admin_port, 30)
        if not up:
            raise RuntimeError(f"proxy did not become ready: {[exit_status(p) for p in proxy_procs]}")
        _trace("healthy")
        if xchg_kind in ("rccl", "tcpbulk"):
            # the bulk executor (RCCL communicator / tcpbulk sockets) formed on this rank before
            # anything is timed: a round-carried final must not fall back to the mesh for want of it
            t_b = time.time()
            while scrape(admin_port).get("qmx_exchange_rccl_active") != 1.0:
                if time.time() - t_b > 90:
                    raise RuntimeError(f"spread: the {xchg_kind} bulk executor did not form in 90 s")
                time.sleep(0.2)
        if dist is not None:
            _barrier(dist, coll_cuda)
        # the reference has no /v1 prefix (oai_proxy.py:959); qmx serves both
        path = "/chat/completions" if args.impl == "reference" and not direct else "/v1/chat/completions"
        warm = {}
        if args.warmup > 0:
            warm = loadgen(bin_dir, proxy_port, args.conns, args.warmup * args.batch, args.lg_threads, args.timeout,
                           spec_path, path, stream)

        def casualties():
            return [dict(exit_status(q), role="mock" if i < len(mock_procs) else "proxy")
                    for i, q in enumerate(mock_procs + proxy_procs) if q.poll() is not None]

        dead_warm = casualties()  # a process that died in warmup fails the run (no silent restart)
        if dead_warm:
            print(f"bench rank {rank}: server process(es) exited during warmup: {dead_warm}", file=sys.stderr,
                  flush=True)
        if dist is not None:
            _barrier(dist, coll_cuda)
        if use_cuda:
            torch.cuda.synchronize()
        scraped = args.impl == "native" and not direct
        m0 = scrape(admin_port) if scraped else {}
        c0 = cpu_snapshot(mock_procs, proxy_procs)
        r0 = rss_mb(proxy_procs[0].pid) if proxy_procs else {}
        g0 = cgroup_cpu_stat()
        t0 = time.perf_counter()
        stats = loadgen(bin_dir, proxy_port, args.conns, args.steps * args.batch, args.lg_threads, args.timeout,
                        spec_path, path, stream)
        if use_cuda:
            torch.cuda.synchronize()
        if dist is not None:
            _barrier(dist, coll_cuda)
        elapsed = time.perf_counter() - t0
        c1 = cpu_snapshot(mock_procs, proxy_procs)
        g1 = cgroup_cpu_stat()
        bd = breakdown(m0, scrape(admin_port), elapsed) if scraped else {}
        bd["pid"] = proxy_procs[0].pid if proxy_procs else None
        bd.update(cpu_breakdown(c0, c1, stats["completed"], elapsed))
        r1 = rss_mb(proxy_procs[0].pid) if proxy_procs else {}
        if r0 and r1:  # rank 0's proxy: resident memory before / after the timed steps, and its peak
            bd["proxy_rss_MB"] = {"start": r0.get("VmRSS"), "end": r1.get("VmRSS"), "peak": r1.get("VmHWM")}
        if g0 and g1:  # the whole job's CPU over the timed region, and any quota throttling
            bd["cgroup"] = {"quota_cpus": g1.get("quota_cpus"),
                            "cores_busy": round((g1.get("usage_usec", 0) - g0.get("usage_usec", 0)) / 1e6 / elapsed, 2)
                            if elapsed else None,
                            "throttled_periods": g1.get("nr_throttled", 0) - g0.get("nr_throttled", 0),
                            "throttled_ms": round((g1.get("throttled_usec", 0) - g0.get("throttled_usec", 0)) / 1e3, 1)}
        dead = casualties()
        if dead and not dead_warm:
            print(f"bench rank {rank}: server process(es) exited during the timed steps: {dead}", file=sys.stderr,
                  flush=True)
        bad = (stats["invalid"] + stats["no_content"] + stats["errors"] + stats["non200"]
               + warm.get("invalid", 0) + warm.get("errors", 0) + warm.get("non200", 0) + len(dead)
               + (args.steps * args.batch - stats["completed"]))
        if args.placement == "spread" and bd.get("exchange"):
            # a remote stream whose delta count disagrees with its worker's, or a worker stream
            # that sent no delta for content it had, is a broken run even if the bytes validated
            bad += int(bd["exchange"]["delta_mismatch"] + bd["exchange"]["worker_nodata"])
        # the harness alone, right after the timed region: the same load generator (connections,
        # threads, validation) straight against this rank's first mock backend, no proxy
        ceiling = None
        if args.ceiling > 0 and not direct and not dead:
            ceiling = harness_ceiling(bin_dir, mock_ports[0], args, mock_procs[0], tmp)
        spread = c3_rows = None
        if (dist is not None and world > 1 and args.spread_check and args.impl == "native"
                and args.placement == "local" and not direct):
            _kill(proxy_procs)  # done measuring; the check brings up its own proxy set
            spread = spread_check(args, SCENARIOS["headline"], rank, world, engine, device, bin_dir, tmp,
                                  mock_ports, dist, n_dev)
            spread_rows = [None] * world
            dist.all_gather_object(spread_rows, spread)
            spread = spread_rows
            c3 = config3_check(args, rank, world, engine, device, bin_dir, tmp, mock_ports, dist, n_dev)
            c3_rows = [None] * world
            dist.all_gather_object(c3_rows, c3)
        local = [elapsed, float(stats["completed"]), float(stats["ttft_p50_ms"]), float(stats["ttft_p99_ms"]),
                 float(stats["errors"] + stats["non200"]), float(stats["ttfb_p50_ms"]), float(stats["lat_p50_ms"]),
                 float(len(dead)), float(stats["invalid"]), float(stats["no_content"]), float(stats["validated"]),
                 float(bad)]
        if dist is not None:
            t = torch.tensor(local, dtype=torch.float64, device="cuda" if coll_cuda else "cpu")
            gathered = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(gathered, t)
            rows = [g.cpu().tolist() for g in gathered]
        else:
            rows = [local]
        headline_ok = all(r[11] == 0 for r in rows)
        # the post-timing checks (spread placement, config 3: other configs than the headline's,
        # each validated response by response) are reported on their own: a failed check is
        # `checks_ok: false` in the JSON line and a warning, not a lost headline measurement
        checks_ok = True
        if spread is not None:
            checks_ok = checks_ok and all(r.get("ok") for r in spread)
        if c3_rows is not None:  # (RCCL not forming is "degraded", still ok: finals took the mesh)
            checks_ok = checks_ok and all((r or {}).get("ok") for r in c3_rows)
        ok = headline_ok
        # per-rank breakdowns, each scraped from that rank's own proxy (admin port)
        bd_rows = [bd]
        ceil_rows = [ceiling]
        if dist is not None:
            bd_rows = [None] * world
            dist.all_gather_object(bd_rows, bd)
            ceil_rows = [None] * world
            dist.all_gather_object(ceil_rows, ceiling)
        if rank == 0:
            max_el = max(r[0] for r in rows)
            total = sum(r[1] for r in rows)
            value = total / max_el
            p50 = statistics.median(r[2] for r in rows)
            baseline = sc["baseline"] if args.impl != "reference" else None
            res = {
                "metric": "proxied req/sec (whole node) + p50 TTFT, 2-backend concatenate stream at 1/2/4/8 GPU"
                          if args.scenario == "headline" else
                          "harness ceiling req/sec (load generator -> mock backend, no proxy) + p50 TTFT" if direct else
                          f"proxied req/sec (whole node) + p50 TTFT, {args.scenario}",
                "value": round(value, 3),
                "unit": "req/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(1000.0 * max_el / args.steps, 3),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": round(value / baseline, 3) if baseline else None,
                "baseline_req_s": baseline,
                "baseline_source": sc.get("baseline_source", BASELINE_SOURCE_SURVEY) if baseline else None,
                "dtype": "bytes (utf-8 SSE text; no float compute)",
                "data": "synthetic: C++ mock backends (role + 4 split <think> fragments + 20 tokens + stop + "
                        "[DONE]) and C++ closed-loop load generator; every response validated against the "
                        "expected event contract",
                "config": {"model": f"{sc['desc']}, skip_final_aggregation={skip_final}",
                           "global_batch": args.batch * world, "seq_len": 26,
                           "parallelism": f"dp{world} (sessions sharded over GPUs: "
                                          + ("each rank's clients on its own port)"
                                             if world > 1 and proxy_port == args.port + RANK_PORT_OFF + rank
                                             else "SO_REUSEPORT)")
                                          + (f" + ep{world} (backend streams spread over ranks, "
                                                f"{xchg_kind.upper()} exchange)"
                                             if args.placement == "spread" and world > 1 else
                                             f" + self spread ({xchg_kind.upper()} rounds to itself)"
                                             if self_spread else ""),
                           "impl": "none (no proxy)" if direct else args.impl,
                           "engine": None if direct else engine if args.impl != "reference" else "reference",
                           "conns_per_rank": args.conns,
                           # hip: io loops post their own ticks into one multi-door grid ("loops",
                           # the default) or hand streams to tick-lane threads ("lanes")
                           "tick_mode": os.environ.get("QMX_TICK_MODE", "auto") if engine == "hip" else None,
                           "io_threads_per_rank": args.threads, "loadgen_threads": args.lg_threads,
                           "mock_threads": args.mock_threads, "cpu_pinning": pinning,
                           # the node's xGMI topology, only when every rank has a GPU of its own
                           # (a rehearsal's ranks share one: no link claim to make)
                           "gpu_links": ({k: v for k, v in link_summary().items() if k != "links_per_gpu"}
                                         if world > 1 and n_dev >= world else None),
                           # rank 0's proxy: HIP streams vs hardware queues per priority level
                           "hip_queues": bd.get("hip_streams"),
                           "self_spread": bool(self_spread) or None},
                "p50_ttft_ms": round(p50, 3),
                "p99_ttft_ms": round(max(r[3] for r in rows), 3),
                "p50_ttfb_ms": round(statistics.median(r[5] for r in rows), 3),
                "p50_latency_ms": round(statistics.median(r[6] for r in rows), 3),
                "errors": int(sum(r[4] for r in rows)),
                # validation: every completed response is checked by the load generator
                "validated": int(sum(r[10] for r in rows)),
                "invalid": int(sum(r[8] for r in rows)),
                "no_content": int(sum(r[9] for r in rows)),
                "processes_exited": int(sum(r[7] for r in rows)),
                "valid": ok,
                "headline_valid": headline_ok,
                "checks_ok": checks_ok,
                "baseline_p50_ttft_ms": sc.get("baseline_ttft_ms"),
                # rank 0's proxy counters over the timed region (SURVEY §5.1 time breakdown),
                # scraped from its own admin port
                "breakdown_one_rank": bd,
            }
            if any(c for c in ceil_rows):
                # what the harness alone sustains on this box (sum over ranks): the proxied number
                # above is only meaningful well below it
                cr = [c for c in ceil_rows if c]
                res["harness_ceiling_req_s"] = round(sum(c["req_s"] for c in cr), 1)
                res["harness_ceiling"] = dict(cr[0], ranks=len(cr)) if len(cr) == 1 else {"per_rank": cr}
            if world > 1:  # every rank's own proxy: distinct pids, its own counters
                res["breakdown_per_rank"] = [compact_breakdown(r, b, row) for r, (b, row) in enumerate(zip(bd_rows, rows))]
            if dead or dead_warm:
                res["exited"] = dead or dead_warm
            if spread is not None:  # outside the timed region; per rank, each from its own proxy
                res["spread_check"] = spread_summary(spread)
            if c3_rows is not None:  # BASELINE config 3, timed on its own (RCCL rounds on a GPU node)
                res["config3"] = config3_summary(c3_rows)
            print(json.dumps(res), flush=True)
    finally:
        _kill(procs)
        if dist is not None:
            dist.destroy_process_group()
    if spread is not None or c3_rows is not None:
        if not checks_ok:
            print("bench: a post-timing check FAILED (spread placement and/or config 3): see 'spread_check' / "
                  "'config3' and 'checks_ok' in the JSON line; the headline measurement is unaffected",
                  file=sys.stderr, flush=True)
    if not ok:
        print("bench: INVALID run (responses failed validation, requests missing, or a server process "
              "exited): see 'invalid' / 'exited' in the JSON line", file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
