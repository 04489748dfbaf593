"""Summarise a rocprofv3 --stats kernel CSV into a markdown table (per update)."""
import csv
import sys


def main(path, updates, title):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", f"source: `{path}` (rocprofv3 --kernel-trace --stats); {updates} updates profiled", "",
           "| kernel | calls/update | avg us | ms/update | % |", "|---|---:|---:|---:|---:|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        name = r["Name"].split("(")[0].replace("void ", "")[:60]
        out.append(f"| `{name}` | {int(r['Calls']) / updates:.1f} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['TotalDurationNs']) / 1e6 / updates:.3f} | {float(r['Percentage']):.1f} |")
    out.append(f"| **total GPU kernel time** | | | **{tot / 1e6 / updates:.2f}** | 100 |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(main(sys.argv[1], float(sys.argv[2]), sys.argv[3]))
