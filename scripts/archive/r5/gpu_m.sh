#!/bin/bash
# round 5 box m: host-side cProfile of the captured LeNet bench loop (per-iteration Python cost)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5m; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/plain.json 2>> $O/err.log || exit 1
ROCKET_BENCH_PROFILE=$O/prof timeout -k 10 180 python bench.py --steps 3000 --warmup 50 > $O/prof.json 2>> $O/err.log || exit 1
python3 - <<PY > $O/host_prof.txt
import pstats, io
s = io.StringIO()
p = pstats.Stats("$O/prof.0", stream=s)
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(45)
print(s.getvalue())
PY
head -120 $O/host_prof.txt
python3 -c "import json;r=json.loads(open('$O/plain.json').read().strip().splitlines()[-1]);print('plain', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'], r['host_ms_p50'])"
