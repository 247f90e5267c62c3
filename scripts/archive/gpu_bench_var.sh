#!/bin/bash
# LeNet bench variance: default-argument runs back to back (what the driver runs), with worst-step stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
S=gpurun_out/summary_var.txt
: > $S
for i in 1 2 3 4 5 6; do
  timeout -k 10 180 python bench.py ${BENCH_ARGS:-} > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err || { echo "bench FAILED" >> $S; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var_$i.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['step_ms_max'],d['step_ms_max_at'],d['host_ms_p50'])" >> $S
done
exit 0
