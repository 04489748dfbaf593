#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches, top kernels).

    python scripts/pmc_summary.py a.csv [b.csv ...]
"""
import collections
import csv
import sys


def main_mem(paths):
    """LDS bank conflicts, MFMA busy and HBM bytes per kernel (per dispatch averages)."""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0][:60]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[(k, p)].add(r.get("Dispatch_Id"))
    order = sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0))[:14]
    print("| kernel | dispatches | LDS bank conflicts / LDS inst | MFMA busy / wave-cycle | "
          "HBM read MB / dispatch | HBM write MB / dispatch |")
    print("|---|---:|---:|---:|---:|---:|")
    for k in order:
        d = tot[k]
        n_c = max(len(nd[(k, paths[0])]), 1)
        n_d = max(len(nd[(k, paths[-1])]), 1)
        lds = d.get("SQ_INSTS_LDS", 0)
        conf = d.get("SQ_LDS_BANK_CONFLICT", 0) / max(lds, 1)
        mfma = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(4 * d.get("SQ_WAVE_CYCLES", 1), 1)
        fetch = d.get("FETCH_SIZE", 0) / n_c / 1024.0      # FETCH_SIZE / WRITE_SIZE are in KB
        write = d.get("WRITE_SIZE", 0) / n_d / 1024.0
        print(f"| `{k}` | {n_c} | {conf:.2f} | {mfma:.3f} | {fetch:.1f} | {write:.1f} |")
    print("\nMFMA busy / wave-cycle = SQ_VALU_MFMA_BUSY_CYCLES / (4 x SQ_WAVE_CYCLES) (wave cycles count quad-cycles); "
          "FETCH_SIZE / WRITE_SIZE are rocprofv3 derived TCC-EA counters (KB).")


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
    if sys.argv[1] == "--mem":
        main_mem(sys.argv[2:])
    else:
        main(sys.argv[1:])
