#!/usr/bin/env python3
"""Per-kernel sums (and per-dispatch means) of every counter in rocprofv3 --pmc counter_collection CSVs.

    python scripts/pmc_dump.py a.csv [b.csv ...] [--top 12] [--match fc_fwd]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in a.csv:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0][:70]
            if a.match and a.match not in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r.get("Dispatch_Id")))
    order = sorted(tot, key=lambda k: -max(tot[k].values()))[: a.top]
    for k in order:
        n = max(1, len(disp[k]) // max(1, len(a.csv)))
        print(f"## `{k}` ({n} dispatches per pass)")
        for c, v in sorted(tot[k].items()):
            print(f"  {c:40s} total {v:16.4g}   per dispatch {v / n:14.4g}")


if __name__ == "__main__":
    main()
