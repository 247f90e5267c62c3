#!/bin/bash
# Per-call conv / BN kernel times of one ResNet-50 step, BN-backward fusion on and off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in 1 0; do
  cd /tmp && ROCKET_BN_BWD_FUSE=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_bnb$mode -o run -- python3 $R/bench.py --model resnet50 --steps 4 --warmup 2 > $R/gpurun_out/prof_bnb$mode.log 2>&1 || exit 1
  cd $R && f=$(find gpurun_out/prof_bnb$mode -name '*kernel_trace.csv' | head -1)
  python3 - "$f" > gpurun_out/bnb_calls_$mode.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "_mt_kernel" in r["Kernel_Name"]]
rows = rows[ends[-2] + 1: ends[-1] + 1]
for r in rows:
    n = r["Kernel_Name"]
    if "conv_kernel" in n or "bn_" in n:
        print(f'{(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:8.1f} {n[:60]}')
PY
  rm -rf gpurun_out/prof_bnb$mode
done
