"""Summarize a rocprofv3 kernel trace over the LAST k training steps (steady state only).

    python bench/summarize_trace.py gpurun_out/prof_x/run_kernel_trace.csv --steps 5 --title "..." > profiles/x.md

Step boundaries are the optimizer launches (adam/sgd multi-tensor kernels); everything MIOpen
benchmarks during its first-use solution search is excluded that way.
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--title", default="kernel profile")
    ap.add_argument("--marker", default="_mt_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} steps in trace")
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
    span = (t1 - t0) / a.steps / 1e3
    print(f"# {a.title}\n")
    print(f"Steady state: last {a.steps} steps of the trace (boundaries = optimizer launches). "
          f"Wall span per step under the profiler: {span:.1f} us; summed kernel time per step: "
          f"{busy / a.steps / 1e3:.1f} us; {len(sel) / a.steps:.1f} kernels per step.\n")
    print("| kernel | calls/step | us/step | share |")
    print("|---|---:|---:|---:|")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"| `{k}` | {n / a.steps:.1f} | {d / a.steps / 1e3:.1f} | {100 * d / busy:.1f}% |")


if __name__ == "__main__":
    main()
