#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, mean counter value per dispatch.

    python tools/pmc_summary.py [--per-tick N] gpurun_out/pmc/*_counter_collection.csv > profiles/<name>.md

--per-tick N: a persistent grid is ONE dispatch serving N ticks (tools/kbench.py --grid prints
grid_ticks); the table then also gives each counter per tick.
"""
import collections
import csv
import sys


import re


def main(argv):
    per_tick = None
    if argv[:1] == ["--per-tick"]:
        per_tick, argv = float(argv[1]), argv[2:]
    paths = argv
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    meta = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])] += 1
            meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"],
                       r["Scratch_Size"])
    kernels = sorted({k for k, _ in agg})
    if per_tick:
        print(f"| kernel | counter | dispatches | mean per dispatch | per tick ({per_tick:.0f} ticks) |")
        print("|---|---|---|---|---|")
    else:
        print("| kernel | counter | dispatches | mean per dispatch |")
        print("|---|---|---|---|")
    for k in kernels:
        for (kk, c) in sorted(agg):
            if kk == k:
                row = f"| {k} | {c} | {cnt[(k, c)]} | {agg[(k, c)] / cnt[(k, c)]:.6g} |"
                if per_tick:
                    row += f" {agg[(k, c)] / per_tick:.6g} |"
                print(row)
    print()
    print("Dispatch geometry as the profiler reports it (its VGPR / SGPR columns are allocation")
    print("granules, not the kernel's register use — see the code-object table below):")
    print()
    print("| kernel | grid | wg | LDS B | VGPR | SGPR | scratch |")
    print("|---|---|---|---|---|---|---|")
    for k in kernels:
        print("| " + k + " | " + " | ".join(meta[k]) + " |")
    res = code_object_resources()
    if res:
        print()
        print("Register use from the in-tree code object (llvm-readelf --notes, AMDHSA metadata):")
        print()
        print("| kernel | VGPRs | SGPRs | SGPR spills (to VGPR lanes) | VGPR spills | scratch B | LDS B |")
        print("|---|---|---|---|---|---|---|")
        for name, r in sorted(res.items()):
            if "qmx_" not in name:
                continue
            m = re.match(r"_ZN3qmx(\d+)", name)  # qmx::<len><name>...
            short = name[m.end():m.end() + int(m.group(1))] if m else name
            print(f"| {short} | {r.get('vgpr_count')} | {r.get('sgpr_count')} | {r.get('sgpr_spill_count')} | "
                  f"{r.get('vgpr_spill_count')} | {r.get('private_segment_fixed_size')} | "
                  f"{r.get('group_segment_fixed_size')} |")


def code_object_resources():
    """{kernel: {field: int}} for the gfx950 code object inside the in-tree extension (the same
    extraction as tests/test_isa.py); {} when the extension or the LLVM tools are missing."""
    import re
    import subprocess
    import tempfile
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    llvm = Path("/opt/rocm/lib/llvm/bin")
    sos = sorted((repo / "quorum_amd").glob("_qmx*.so"))
    if not sos or not (llvm / "llvm-readelf").exists():
        return {}
    try:
        with tempfile.TemporaryDirectory() as d:
            fat, co = Path(d) / "fat.bin", Path(d) / "dev.co"
            subprocess.run([str(llvm / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(sos[0]),
                            str(Path(d) / "host.so")], check=True, capture_output=True)
            targets = subprocess.run([str(llvm / "clang-offload-bundler"), "--list", "--type=o", f"--input={fat}"],
                                     check=True, capture_output=True, text=True).stdout.split()
            gfx = [t for t in targets if t.endswith("gfx950")]
            if not gfx:
                return {}
            subprocess.run([str(llvm / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                            f"--targets={gfx[0]}", f"--output={co}"], check=True, capture_output=True)
            notes = subprocess.run([str(llvm / "llvm-readelf"), "--notes", str(co)], check=True,
                                   capture_output=True, text=True).stdout
    except (OSError, subprocess.CalledProcessError):
        return {}
    out, cur = [], None
    for line in notes.splitlines():
        if re.match(r"\s*-\s+\.", line):
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
        if m:
            cur["name"] = m.group(1)
            continue
        m = re.match(r"\s*-?\s*\.(private_segment_fixed_size|vgpr_count|vgpr_spill_count|sgpr_count|sgpr_spill_count|"
                     r"group_segment_fixed_size):\s+(\d+)", line)
        if m:
            cur[m.group(1)] = int(m.group(2))
    return {d["name"]: d for d in out if "name" in d}


if __name__ == "__main__":
    main(sys.argv[1:])
