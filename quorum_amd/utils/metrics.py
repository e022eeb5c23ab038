"""Per-rank metrics in Prometheus text format (SURVEY §5.5 — absent in the reference).

Counters/histograms are plain module-level state (one process = one rank); the
``/metrics`` endpoint renders them.  Nothing here touches the hot path beyond a few
integer adds.
"""
from __future__ import annotations

import threading
from collections import defaultdict
from typing import Dict, List, Tuple

_lock = threading.Lock()
_counters: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], float] = defaultdict(float)

# latency histogram buckets (seconds)
_BUCKETS = [0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0]


class Histogram:
    def __init__(self, name: str, help_: str):
        self.name = name
        self.help = help_
        self.counts = [0] * (len(_BUCKETS) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        i = 0
        while i < len(_BUCKETS) and v > _BUCKETS[i]:
            i += 1
        self.counts[i] += 1
        self.sum += v
        self.n += 1

    def render(self) -> List[str]:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} histogram"]
        cum = 0
        for b, c in zip(_BUCKETS, self.counts):
            cum += c
            out.append(f'{self.name}_bucket{{le="{b}"}} {cum}')
        cum += self.counts[-1]
        out.append(f'{self.name}_bucket{{le="+Inf"}} {cum}')
        out.append(f"{self.name}_sum {self.sum}")
        out.append(f"{self.name}_count {self.n}")
        return out


HIST = {
    "ttft": Histogram("qmx_ttft_seconds", "time from request to first content event"),
    "request": Histogram("qmx_request_seconds", "request latency"),
    "upstream": Histogram("qmx_upstream_seconds", "upstream call latency"),
    "tick": Histogram("qmx_tick_seconds", "engine tick wall time"),
}


def inc(name: str, value: float = 1.0, **labels: str) -> None:
    key = (name, tuple(sorted(labels.items())))
    with _lock:
        _counters[key] += value


def observe(hist: str, value: float) -> None:
    with _lock:
        HIST[hist].observe(value)


def observe_tick(seconds: float, n_slots: int) -> None:
    with _lock:
        HIST["tick"].observe(seconds)
        _counters[("qmx_tick_slots_total", ())] += n_slots
        _counters[("qmx_ticks_total", ())] += 1


def render() -> str:
    lines: List[str] = []
    with _lock:
        for (name, labels), v in sorted(_counters.items()):
            lab = ",".join(f'{k}="{val}"' for k, val in labels)
            lines.append(f"{name}{{{lab}}} {v}" if lab else f"{name} {v}")
        for h in HIST.values():
            lines.extend(h.render())
    return "\n".join(lines) + "\n"


def reset() -> None:
    with _lock:
        _counters.clear()
        for k, h in list(HIST.items()):
            HIST[k] = Histogram(h.name, h.help)
