#!/bin/bash
# Kernel trace of the captured LeNet step (steady state), summarized on the box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_lenet -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/prof_lenet.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_lenet -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 50 --marker mlp3_wgrad_kernel --title "LeNet bs1024 fused step (captured, launch-list replay; AdamW fused into the wgrad launch), 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/lenet_graph_kernels.md; rc=$?
python3 - "$f" > gpurun_out/lenet_graph_gaps.txt <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-4 * 50:]
prev = None
gaps = {}
for r in rows:
    s, e, n = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]
    if prev is not None:
        gaps.setdefault(n, []).append((s - prev) / 1e3)
    prev = e
for n, g in gaps.items():
    print(f"{n:42s} gap before (us) median {statistics.median(g):6.2f}")
PY
rm -rf gpurun_out/prof_lenet
exit $rc
