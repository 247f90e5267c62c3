#!/bin/bash
# kernel-trace durations of single GEMM runs: CASES="shape:engine ..." -> gpurun_out/r6kt/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6kt; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for case in ${CASES:-proj:x5 proj:lib}; do
  shp=${case%%:*}; eng=${case#*:}; tag=${shp}_${eng//:/_}
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 $R/bench/x5_one.py $shp $eng 6 > $O/$tag.log 2>&1 || { echo "trace $case failed"; tail -5 $O/$tag.log; exit 1; }
  python3 - $O/$tag "$case" >> $O/summary.txt <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "xgemm" in n or "Cijk" in n or "gemm" in n.lower():
            d[n[:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    v = v[2:] or v
    print(sys.argv[2], n, "calls", len(v), "median_us", round(sorted(v)[len(v) // 2], 2))
PY
  rm -rf $O/$tag
done
cat $O/summary.txt
