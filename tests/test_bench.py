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
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
