#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches, top kernels).

    python scripts/pmc_summary.py a.csv [b.csv ...]
"""
import collections
import csv
import sys


def main(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0][:60]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r.get("Dispatch_Id")))
    order = sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0))[:14]
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "TCC_HIT_sum", "TCC_MISS_sum"]
    print("| kernel | per-wave VALU | MFMA | SALU | LDS | VMEM rd | VMEM wr | wait_any | wait_inst | active | "
          "L2 hit |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in order:
        d = tot[k]
        w = max(d.get("SQ_WAVES", 1), 1)
        wc = max(d.get("SQ_WAVE_CYCLES", 1), 1)
        hit = d.get("TCC_HIT_sum", 0)
        miss = d.get("TCC_MISS_sum", 0)
        print(f"| `{k}` | {d.get('SQ_INSTS_VALU', 0) / w:.0f} | {d.get('SQ_INSTS_MFMA', 0) / w:.0f} | "
              f"{d.get('SQ_INSTS_SALU', 0) / w:.0f} | {d.get('SQ_INSTS_LDS', 0) / w:.0f} | "
              f"{d.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | {d.get('SQ_INSTS_VMEM_WR', 0) / w:.0f} | "
              f"{d.get('SQ_WAIT_ANY', 0) / wc:.2f} | {d.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | "
              f"{d.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} | {hit / max(hit + miss, 1):.2f} |")
    print("\nper-wave = instructions per wave; wait_any / wait_inst / active = fractions of wave cycles "
          "(SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES); L2 hit = TCC_HIT/(HIT+MISS).")


if __name__ == "__main__":
    main(sys.argv[1:])
