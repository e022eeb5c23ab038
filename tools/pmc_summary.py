#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, mean counter value per dispatch.

    python tools/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv > profiles/<name>.md
"""
import collections
import csv
import sys


def main(paths):
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
    print("| kernel | counter | dispatches | mean per dispatch |")
    print("|---|---|---|---|")
    for k in kernels:
        for (kk, c) in sorted(agg):
            if kk == k:
                print(f"| {k} | {c} | {cnt[(k, c)]} | {agg[(k, c)] / cnt[(k, c)]:.6g} |")
    print()
    print("| kernel | grid | wg | LDS B | VGPR | SGPR | scratch |")
    print("|---|---|---|---|---|---|---|")
    for k in kernels:
        print("| " + k + " | " + " | ".join(meta[k]) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
