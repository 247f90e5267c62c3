#!/bin/bash
# ViT-B/16 x5-mode kernel sequence of one traced step (GEMM-related kernels, in order) -> gpurun_out/r6vs/seq.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6vs; mkdir -p $O; rm -rf $O/t
cd /tmp && export TMPDIR=/tmp
ROCKET_VIT_GEMM=${MODE:-x5} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 $R/bench.py --model vit_b16 --steps 3 --warmup 2 > $O/run.log 2>&1 || { echo "trace failed"; tail -20 $O/run.log; exit 1; }
python3 - $O/t > $O/seq_${MODE:-x5}.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last adam_mt marks step ends: print the kernels of the last full step
ends = [i for i, r in enumerate(rows) if "adam_mt" in r["Kernel_Name"]]
seg = rows[ends[-2] + 1: ends[-1] + 1]
for r in seg:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    gr = r.get("Grid_Size", "")
    print(f"{d:8.1f} us grid {gr:>8} {n[:100]}")
PY
rm -rf $O/t
head -5 $O/seq_${MODE:-x5}.txt
