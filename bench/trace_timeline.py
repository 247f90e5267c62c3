"""Print the last kernels of a rocprofv3 kernel-trace CSV as a timeline (start / end relative to
the first printed kernel, gap to the previous kernel's end) — for checking which launches overlap.

    python bench/trace_timeline.py <kernel_trace.csv> [--last 12]
"""

import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=12)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    rows = rows[-a.last:]
    t0 = rows[0][0]
    prev_end = None
    for s, e, n in rows:
        gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:7.2f}"
        print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} dur {(e - s) / 1e3:6.2f} gap {gap:>7}  {n}")
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
