#!/usr/bin/env python3
"""Symbolise and summarise a qmx CPU profile (QMX_PROF=<path>, csrc/qmx_prof.h).

    python tools/cpuprof.py gpurun_out/prof/cpu.1234.txt [--top 40] [--json out.json]

Reports where the data plane's CPU goes: self time by function (innermost frame), by
category (socket writes / reads, epoll, locks + wakeups, allocator, memcpy, HTTP / JSON,
engine host work, HIP runtime), and inclusive time of qmx functions.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import shutil
import subprocess
import sys

SYMBOLIZER = shutil.which("llvm-symbolizer") or "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
CATEGORIES = [
    ("socket write", r"^(__libc_)?(send|sendmsg|sendto|write|writev)$|__send|__write"),
    ("socket read", r"^(__libc_)?(recv|recvmsg|recvfrom|read|readv)$|__recv|__read"),
    ("epoll", r"epoll_wait|epoll_ctl|epoll_pwait"),
    ("locks/wakeups", r"futex|pthread_mutex|pthread_cond|__lll_lock|sched_yield|condition_variable|nanosleep"),
    ("accept/close/socket", r"accept|^close$|__close|socket|setsockopt|connect"),
    ("allocator", r"malloc|free|operator new|operator delete|_int_malloc|_int_free|realloc|cfree"),
    ("memcpy/memmove/memset", r"memcpy|memmove|memset|memchr|memmem|memcmp|strlen"),
    ("HIP runtime", r"^hip|amd::|^roc|hsa_|^Hip|libamdhip64|libhsa"),
    ("json", r"json|JVal|py_float_repr"),
    ("engine host", r"HostEngine|CpuEngine|HipEngine|process_slot|filter_feed|classify|escape|strip_final|finalize"),
    ("http/proxy", r"qmx::|Loop::|Session|http|parse"),
]


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local_module(mod: str) -> str:
    """A profile taken on the GPU box names modules under its own repo copy: map our own
    binaries back to this tree (they are the same files — the box runs the shipped .so)."""
    if os.path.exists(mod):
        return mod
    base = os.path.basename(mod)
    for cand in (os.path.join(ROOT, "quorum_amd", base), os.path.join(ROOT, "quorum_amd", "bin", base)):
        if os.path.exists(cand):
            return cand
    return mod


def symbolize(frames):
    by_mod = collections.defaultdict(set)
    for fr in frames:
        mod, _, off = fr.rpartition("+")
        by_mod[mod].add(off)
    names = {}
    for mod0, offs in by_mod.items():
        offs = sorted(offs)
        mod = local_module(mod0)
        if mod in ("?", "") or not shutil.which(SYMBOLIZER) and not SYMBOLIZER.startswith("/"):
            for o in offs:
                names[f"{mod0}+{o}"] = f"{mod0}+{o}"
            continue
        try:
            out = subprocess.run([SYMBOLIZER, f"--obj={mod}", "-C", "--no-inlines", "--functions=linkage"],
                                 input="\n".join(offs) + "\n", capture_output=True, text=True, timeout=300).stdout
        except (OSError, subprocess.SubprocessError):
            out = ""
        blocks = [b.splitlines() for b in out.strip().split("\n\n")] if out.strip() else []
        short = mod.rsplit("/", 1)[-1]
        for o, blk in zip(offs, blocks + [[]] * (len(offs) - len(blocks))):
            fn = blk[0] if blk else "??"
            names[f"{mod0}+{o}"] = f"{fn} [{short}]" if fn != "??" else f"?? [{short}+{o}]"
    return names


def category(fn: str) -> str:
    base = fn.split(" [")[0]
    for cat, rx in CATEGORIES:
        if re.search(rx, base):
            return cat
    lib = fn.rsplit("[", 1)[-1]
    return "other (" + lib.split("+")[0].rstrip("]") + ")"


def summarize(path: str, top: int = 40):
    stacks = []
    with open(path) as f:
        for ln in f:
            if ln.startswith("#") or not ln.strip():
                continue
            stacks.append(ln.strip().split(";"))
    names = symbolize({fr for st in stacks for fr in st})
    n = len(stacks)
    self_c = collections.Counter()
    cat_c = collections.Counter()
    incl = collections.Counter()
    callers = collections.defaultdict(collections.Counter)  # category -> first qmx frame above it
    for st in stacks:
        fns = [names.get(fr, fr) for fr in st]
        # drop the handler and the sigreturn trampoline above the interrupted frame
        h = next((i for i, x in enumerate(fns) if "on_prof" in x), None)
        if h is not None:
            fns = fns[h + 2:]
        if not fns:
            continue
        self_c[fns[0]] += 1
        # the category of a sample = the innermost frame that matches one (libc wrappers first)
        cats = [category(x) for x in fns]
        cat = next((c for c in cats if not c.startswith("other")), cats[0])
        cat_c[cat] += 1
        own = next((x for x in fns if "[_qmx" in x or "[qmx_" in x), None)
        if own is not None and own != fns[0]:
            callers[cat][own.split(" [")[0]] += 1
        for x in set(fns):
            if "qmx" in x or "Loop" in x:
                incl[x] += 1
    pct = lambda c: round(100.0 * c / max(n, 1), 2)  # noqa: E731
    return {"samples": n,
            "by_category_pct": {k: pct(v) for k, v in cat_c.most_common()},
            "self_top_pct": {k: pct(v) for k, v in self_c.most_common(top)},
            "inclusive_qmx_pct": {k: pct(v) for k, v in incl.most_common(top)},
            # which of our functions issued the library time of each category
            "callers_pct": {c: {k: pct(v) for k, v in cc.most_common(12)} for c, cc in callers.items()}}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("profiles", nargs="+")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    ap.add_argument("--callers", action="append", default=[],
                    help="print our functions that issued a category's time (e.g. allocator)")
    a = ap.parse_args(argv)
    res = {p: summarize(p, a.top) for p in a.profiles}
    for p, r in res.items():
        print(f"== {p}: {r['samples']} samples")
        print("-- by category (%)")
        for k, v in r["by_category_pct"].items():
            print(f"  {v:6.2f}  {k}")
        print("-- self (%)")
        for k, v in list(r["self_top_pct"].items())[:a.top]:
            print(f"  {v:6.2f}  {k}")
        for cat in a.callers:
            print(f"-- callers of {cat} (%)")
            for k, v in r["callers_pct"].get(cat, {}).items():
                print(f"  {v:6.2f}  {k[:150]}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
