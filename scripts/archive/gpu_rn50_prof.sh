#!/bin/bash
# ResNet-50 steady-state kernel trace (native convs) -> gpurun_out/rn50_kernels.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_rn50 -o run -- python3 $R/bench.py --model ${MODEL:-resnet50} --steps 4 --warmup 2 > $R/gpurun_out/prof_rn50.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_rn50 -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 3 --title "${MODEL:-resnet50} bf16 native convs - rocprofv3 --kernel-trace" > gpurun_out/rn50_kernels.md
python3 - "$f" > gpurun_out/rn50_conv_calls.txt <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "_mt_kernel" in r["Kernel_Name"]]
rows = rows[ends[-2] + 1: ends[-1] + 1]
for r in rows:
    n = r["Kernel_Name"]
    if "conv_kernel" in n or "igemm" in n or "ck::" in n or "reduce" in n:
        print(f'{(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:8.1f} us grid={r.get("Grid_Size")} {n[:70]}')
PY
rm -rf gpurun_out/prof_rn50
