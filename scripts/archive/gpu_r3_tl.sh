#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r3t; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 300 --warmup 20 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
f=$(find $O/tr -name '*kernel_trace.csv' | head -1)
cd $R && python3 bench/trace_timeline.py "$f" --last 14 > $O/timeline.txt && cat $O/timeline.txt
rm -rf $O/tr
