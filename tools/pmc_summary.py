#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, mean counter value per dispatch.

    python tools/pmc_summary.py [--per-tick N] gpurun_out/pmc/*_counter_collection.csv > profiles/<name>.md

--per-tick N: a persistent grid is ONE dispatch serving N ticks (tools/kbench.py --grid prints
grid_ticks); the table then also gives each counter per tick.
"""
import collections
import csv
import sys


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
    print("| kernel | grid | wg | LDS B | VGPR | SGPR | scratch |")
    print("|---|---|---|---|---|---|---|")
    for k in kernels:
        print("| " + k + " | " + " | ".join(meta[k]) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
