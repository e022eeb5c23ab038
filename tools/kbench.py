#!/usr/bin/env python3
"""Tick-kernel microbenchmark: one tick over N slots of the benchmark's upstream stream shape.

    QMX_STAGE_TIMING=1 python tools/kbench.py [--slots 1,16,256] [--iters 50]

Prints per-configuration host wall time per tick, GPU kernel time and (with
QMX_STAGE_TIMING=1) the per-stage wall-time split measured in-kernel with s_memrealtime.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mock_stream(tokens=20, think=True):
    def ev(delta, finish="null"):
        return ('data: {"id": "chatcmpl-mock", "object": "chat.completion.chunk", "created": 1700000000, '
                '"model": "mock", "choices": [{"index": 0, "delta": %s, "finish_reason": %s}]}\n\n'
                % (delta, finish)).encode()
    out = [ev('{"role": "assistant", "content": ""}')]
    if think:
        out += [ev('{"content": "<thi"}'), ev('{"content": "nk>let me reason about the request"}'),
                ev('{"content": " carefully before answering</th"}'), ev('{"content": "ink>"}')]
    words = ["The", " quick", " brown", " fox", " jumps", " over", " the", " lazy", " dog", "."]
    out += [ev('{"content": "%s"}' % words[i % 10]) for i in range(tokens)]
    out += [ev("{}", '"stop"'), b"data: [DONE]\n\n"]
    return b"".join(out)


def tagdense_stream(tokens=20):
    """Tag-dense content (markup / code the filter must scan: every token has '<' bytes —
    real tags, near misses, comparisons, nested think blocks): the shape where the MFMA
    matcher does the work (one v_mfma_i32_16x16x64_i8 per 16 '<' candidates)."""
    def ev(delta, finish="null"):
        return ('data: {"id": "chatcmpl-mock", "object": "chat.completion.chunk", "created": 1700000000, '
                '"model": "mock", "choices": [{"index": 0, "delta": %s, "finish_reason": %s}]}\n\n'
                % (delta, finish)).encode()
    pieces = ["<div><b>x</b> <think>a<reason>b</reason>c</think> y",
              " if (a < b && c <d) <thin> <thought>t</thought> ",
              "<reasoning>r</REASONING> <Think>z</THINK> <th", "ink>k</think> <table><tr><td>1</td></tr>",
              " <thoughts> <reason-> <reasonin> </ <<think>q</think>>"]
    out = [ev('{"role": "assistant", "content": ""}')]
    out += [ev('{"content": "%s"}' % pieces[i % len(pieces)]) for i in range(tokens)]
    out += [ev("{}", '"stop"'), b"data: [DONE]\n\n"]
    return b"".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", default="1,16,64,256,1024")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--engine", default="hip")
    ap.add_argument("--grid", type=int, default=0,
                    help="N > 0: post the ticks into door 0 of an N-door persistent grid (HipGrid, the loop-tick "
                         "production kernel qmx_tick_persistent) instead of one-shot launches")
    ap.add_argument("--combos", default="ft,f,t",
                    help="(filter, emit) combinations: ft = filter+emit, f = filter only, t = emit only")
    ap.add_argument("--shape", default="mock", choices=["mock", "tagdense"],
                    help="mock: the benchmark's upstream stream; tagdense: '<'-heavy content (MFMA matcher load)")
    ap.add_argument("--events-per-tick", type=int, default=0,
                    help="stream the body N events per tick (steady-state serving shape); 0 = whole body in one tick")
    args = ap.parse_args()
    from quorum_amd.ops.native import NativeEngine

    body = mock_stream() if args.shape == "mock" else tagdense_stream()
    tags = ["think", "reason", "reasoning", "thought"]
    results = []
    grid = None
    if args.grid > 0:
        from quorum_amd.ops import native

        grid = native.require().HipGrid(0, args.grid, 8)
    combos = {"ft": (True, True), "f": (True, False), "t": (False, True)}
    for filt, emit in [combos[c] for c in args.combos.split(",")]:
        for n in [int(x) for x in args.slots.split(",")]:
            kw = {"grid": grid, "door": 0} if grid is not None else {}
            eng = NativeEngine(args.engine, tags, device=0, max_slots=4096, content_cap=1 << 16, **kw)
            walls = []
            evs = [e + b"\n\n" for e in body.split(b"\n\n") if e]
            k = args.events_per_tick or len(evs)
            pieces = [b"".join(evs[i:i + k]) for i in range(0, len(evs), k)]
            for it in range(args.iters):
                slots = [eng.open(i % 8, filt, emit) for i in range(n)]
                for pi, piece in enumerate(pieces):
                    for s in slots:
                        eng.feed(s, piece)
                        if pi == len(pieces) - 1:
                            eng.finish(s)
                    t0 = time.perf_counter()
                    res, _ = eng.tick(1700000000)
                    walls.append(time.perf_counter() - t0)
                for s in slots:
                    eng.release(s)
            st = eng._e.kernel_stats() if args.engine == "hip" else {}
            walls.sort()
            rec = {"filter": filt, "emit": emit, "shape": args.shape, "slots": n, "bytes_per_slot": len(body),
                   "events_per_tick": k,
                   "wall_us_p50": round(1e6 * walls[len(walls) // 2], 1),
                   "wall_us_min": round(1e6 * walls[0], 1)}
            if st:
                rec["kernel_us_avg"] = round(1000 * st["kernel_ms"] / max(st["launches"], 1), 1)
                if st.get("stage_items"):
                    ni = st["stage_items"]
                    rec["stage_us_per_item"] = {k: round(v / ni, 2) for k, v in st.items()
                                                if k.startswith("stage") and k.endswith("_us")}
                rec["shader_mhz"] = round(st.get("shader_mhz", 0), 1)
                if st.get("s3_events"):
                    rec["s3_per_item"] = {k: round(st[k] / st["stage_items"], 2)
                                          for k in ("s3_events", "s3_full_parses", "s3_template_hits", "s3_hole_hits",
                                                    "s3_cycles_full", "s3_cycles_template", "s3_cycles_lex", "s3_cycles_hole",
                                                    "s3a_unresolved")
                                          if k in st}
                rec["MB_per_s"] = round(n * len(body) / len(pieces) / (st["kernel_ms"] / max(st["launches"], 1)) / 1e3, 1)
            if grid is not None:
                rec["grid_ticks"] = st.get("grid_ticks")
                rec["grid_launches"] = st.get("grid_launches")
            results.append(rec)
            print(json.dumps(rec), flush=True)
    if grid is not None:  # the grid's one dispatch ends here: its counters cover every tick above
        grid.stop()
        print(json.dumps({"grid_stats": grid.stats()}), flush=True)
    return results


if __name__ == "__main__":
    main()
