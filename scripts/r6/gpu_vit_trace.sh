#!/bin/bash
# ViT-B/16 kernel-trace stats per GEMM mode -> gpurun_out/r6vt/<mode>.txt (top kernels by total time)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6vt; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mode in ${MODES:-lib x5}; do
  ROCKET_VIT_GEMM=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$mode -o run -- python3 $R/bench.py --model vit_b16 --steps 6 --warmup 3 > $O/$mode.log 2>&1 || { echo "trace $mode failed"; tail -20 $O/$mode.log; exit 1; }
  python3 - $O/$mode $mode > $O/$mode.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {sys.argv[2]}: {len(rows)} kernels, total {tot/1e6:.2f} ms over the traced steps (warmup+timed)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.3f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% calls {r["Calls"]:>5} avg {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:110]}')
PY
  rm -rf $O/$mode
  cat $O/$mode.txt
done
