"""Merge rocprofv3 ``--pmc`` passes of one workload into a per-kernel counter table (Markdown).

    python bench/summarize_pmc.py gpurun_out/pmc/lenet_A gpurun_out/pmc/lenet_B ... \
        --steps 3 --title "LeNet step" > profiles/r1_pmc_lenet.md

Every pass is a separate run of the same program; each pass is reduced to per-kernel means over
the dispatches of its LAST ``--steps`` training steps (step boundary = the optimizer kernel,
``--marker``), so warm-up, MIOpen solution search and the untimed steps are excluded.  Derived:

* ``active/wait/inst-stall`` — SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY, SQ_WAIT_INST_ANY as shares of
  SQ_WAVE_CYCLES (they partition it);
* ``MFMA util`` — SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCD x 256 CU x 4 SIMD).
  GRBM_GUI_ACTIVE is accumulated over the 8 XCDs (without the /8 the hipBLASLt ViT GEMMs, which
  run at ~0.8-1 PFLOP/s by their FLOP count, would read 3-5 %);
* ``LDS conflict`` — SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``HBM GB/s`` — (FETCH_SIZE + WRITE_SIZE) KiB / kernel time (FETCH_SIZE under-counts wide
  streams by up to 2x on gfx950, see MI355X_MICROARCH.md §HBM: a lower bound).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

CUS, SIMDS, XCDS = 256, 4, 8


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:80]


def load_pass(d: str, marker: str, steps: int):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None, None
    per = collections.defaultdict(dict)  # dispatch -> {name, ctr: value, dur}
    for f in files:
        for r in csv.DictReader(open(f)):
            did = (f, int(r["Dispatch_Id"]))
            e = per[did]
            e["name"] = r["Kernel_Name"]
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                e["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e["grid"] = r.get("Grid_Size")
            e["wg"] = r.get("Workgroup_Size")
            e["lds"] = r.get("LDS_Block_Size")
            e["vgpr"] = r.get("VGPR_Count") or r.get("Arch_VGPR_Count")
            e["agpr"] = r.get("Accum_VGPR_Count")
    order = sorted(per)
    marks = [i for i, k in enumerate(order) if marker in per[k]["name"]]
    if len(marks) >= steps + 1:
        order = order[marks[-steps - 1] + 1 : marks[-1] + 1]
        nsteps = steps
    else:
        nsteps = max(1, len(marks))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for k in order:
        e = per[k]
        n = short(e["name"])
        a = agg[n]
        a["calls"] += 1
        for c, v in e.items():
            if isinstance(v, (int, float)):
                a[c] += v
        meta[n] = (e.get("grid"), e.get("wg"), e.get("lds"), e.get("vgpr"), e.get("agpr"))
    return agg, (meta, nsteps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passes", nargs="+")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="_mt_kernel")
    ap.add_argument("--title", default="PMC counters")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    merged = collections.defaultdict(lambda: collections.defaultdict(float))
    meta, nsteps = {}, a.steps
    for d in a.passes:
        agg, m = load_pass(d, a.marker, a.steps)
        if agg is None:
            continue
        meta.update(m[0])
        nsteps = m[1]
        for n, cs in agg.items():
            calls = cs["calls"]
            for c, v in cs.items():
                if c == "calls":
                    merged[n]["calls"] = max(merged[n]["calls"], calls)
                else:
                    key = c if c != "dur_ns" else "dur_ns"
                    # per-call mean, averaged over passes that measured it
                    merged[n].setdefault("_n_" + key, 0.0)
                    merged[n]["_n_" + key] += 1
                    merged[n][key] += v / calls
    rows = []
    for n, cs in merged.items():
        m = {k: (v / cs["_n_" + k] if ("_n_" + k) in cs else v) for k, v in cs.items() if not k.startswith("_n_")}
        m["us_step"] = m.get("dur_ns", 0.0) * m["calls"] / nsteps / 1e3
        rows.append((n, m))
    rows.sort(key=lambda r: -r[1]["us_step"])
    tot = sum(m["us_step"] for _, m in rows) or 1.0
    print(f"# {a.title}\n")
    print(f"rocprofv3 --kernel-trace --pmc, {len(a.passes)} passes (one run each), per-kernel means over the last "
          f"{nsteps} steps.  Times are from the counter runs (kernels serialised by the profiler).\n")
    print("| kernel | calls/step | us/call | share | grid/wg | VGPR/AGPR/LDS | active/wait/inst-stall % | VALU/LDS/MFMA inst per wave | MFMA util % | LDS bank-conflict % | HBM GB/s | L2 hit % |")
    print("|---|---:|---:|---:|---|---|---|---|---:|---:|---:|---:|")
    for n, m in rows[: a.top]:
        g = meta.get(n, (None,) * 5)
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        part = "/".join(f"{100 * m.get(c, 0) / wc:.0f}" for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")) if wc else "-"
        waves = m.get("SQ_WAVES", 0.0)
        inst = "/".join(f"{m.get(c, 0) / waves:.0f}" for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA")) if waves else "-"
        ga = m.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (ga / XCDS * CUS * SIMDS):.1f}" if ga and "SQ_VALU_MFMA_BUSY_CYCLES" in m else "-"
        lds = f"{100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1f}" if m.get("SQ_LDS_IDX_ACTIVE") else "-"
        dur = m.get("dur_ns", 0.0)
        hbm = "-"
        if dur and ("FETCH_SIZE" in m or "WRITE_SIZE" in m):
            hbm = f"{(m.get('FETCH_SIZE', 0) + m.get('WRITE_SIZE', 0)) * 1024 / dur:.0f}"
        hit = "-"
        if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0):
            hit = f"{100 * m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.0f}"
        print(f"| `{n}` | {m['calls'] / nsteps:.1f} | {dur / 1e3:.1f} | {100 * m['us_step'] / tot:.1f}% | {g[0]}/{g[1]} | "
              f"{g[3]}/{g[4]}/{g[2]} | {part} | {inst} | {mfma} | {lds} | {hbm} | {hit} |")


if __name__ == "__main__":
    main()
