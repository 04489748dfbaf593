"""Per-kernel summary of the steady-state window of a rocprofv3 kernel trace (bench.py --prof-window).

Only dispatches between the two ``prof_window_marker_kernel`` launches count: setup, warm-up, graph capture
and the post-window bookkeeping are excluded, so the table sums to the timed updates' GPU time.

    python scripts/prof_window.py <kernel_trace.csv> <updates in the window> <title>
"""
import csv
import os
import statistics
import sys
from collections import defaultdict


def main(path, updates, title):
    rows = list(csv.DictReader(open(path)))
    key = next(k for k in rows[0] if k.lower().replace("_", "") in ("kernelname", "name"))
    t0k = next(k for k in rows[0] if "start" in k.lower())
    t1k = next(k for k in rows[0] if "end" in k.lower())
    rows.sort(key=lambda r: int(r[t0k]))
    marks = [int(r[t0k]) for r in rows if "prof_window_marker" in r[key]]
    if len(marks) < 2:
        raise SystemExit("no prof_window markers in the trace (run bench.py --prof-window)")
    lo, hi = marks[0], marks[-1]
    # PROF_BY_GRID=1: separate dispatches of one kernel by grid size (e.g. the fc1 and fc2 launches of a template)
    gkey = next((k for k in rows[0] if k.lower().replace("_", "") == "gridsize"), None)
    by_grid = os.environ.get("PROF_BY_GRID") == "1" and gkey is not None
    tot = defaultdict(float)
    calls = defaultdict(int)
    durs = defaultdict(list)
    for r in rows:
        t = int(r[t0k])
        if lo < t < hi and "prof_window_marker" not in r[key]:
            name = r[key].split("(")[0].replace("void ", "")
            if by_grid:
                name += f" [grid {r[gkey]}]"
            tot[name] += int(r[t1k]) - t
            calls[name] += 1
            durs[name].append((int(r[t1k]) - t) / 1e3)
    total = sum(tot.values())
    # busy time = union of the window's dispatch intervals: below the summed kernel time when launches of
    # different streams (the split rollout's path groups) overlap
    iv = sorted((int(r[t0k]), int(r[t1k])) for r in rows
                if lo < int(r[t0k]) < hi and "prof_window_marker" not in r[key])
    busy, cur0, cur1 = 0, None, None
    for a, b in iv:
        if cur1 is None or a > cur1:
            if cur1 is not None:
                busy += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        busy += cur1 - cur0
    out = [f"# {title}", "", f"source: `{path}` (rocprofv3 --kernel-trace); {updates} timed updates between the "
           f"bench.py --prof-window markers; wall between markers {(hi - lo) / 1e6 / updates:.3f} ms per update", "",
           "| kernel | calls/update | avg us | min / median / max us | ms/update | % |",
           "|---|---:|---:|---:|---:|---:|"]
    for name in sorted(tot, key=lambda n: -tot[n])[:30]:
        out.append(f"| `{name[:70] if not by_grid else name[:50] + name[name.rfind(' ['):]}` | {calls[name] / updates:.1f} | {tot[name] / calls[name] / 1e3:.1f} | "
                   f"{min(durs[name]):.1f} / {statistics.median(durs[name]):.1f} / {max(durs[name]):.1f} | "
                   f"{tot[name] / 1e6 / updates:.3f} | {100 * tot[name] / total:.1f} |")
    out.append(f"| **total GPU kernel time** | | | | **{total / 1e6 / updates:.2f}** | 100 |")
    out.append(f"| **GPU busy (union of dispatch intervals)** | | | | **{busy / 1e6 / updates:.2f}** | "
               f"{100 * busy / max(total, 1):.0f} |")
    seq = os.environ.get("PROF_SEQ")
    if seq:
        # PROF_SEQ=<substring>: the durations of the matching kernel in dispatch order (per-step patterns), with the
        # kernel that ran just before each call
        prev, lines = None, []
        for r in rows:
            t = int(r[t0k])
            if not (lo < t < hi) or "prof_window_marker" in r[key]:
                continue
            nm = r[key].split("(")[0].replace("void ", "")
            if seq in nm:
                lines.append(f"{(int(r[t1k]) - t) / 1e3:.1f} after {prev[:40] if prev else '-'}")
            prev = nm
        out.append("")
        out.append(f"dispatch-order durations (us) of `{seq}`: " + "; ".join(lines[:84]))
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(main(sys.argv[1], float(sys.argv[2]), sys.argv[3]))
