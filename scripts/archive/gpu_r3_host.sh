#!/bin/bash
# LeNet host-side cost: plain run (host_issue_ms / host_ms_p50) + cProfile of a long run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3h; export TMPDIR=/tmp
O=$R/gpurun_out/r3h
timeout -k 10 200 python bench.py --steps 2000 --warmup 20 > $O/lenet_2000.json 2>$O/lenet_2000.err || { tail -20 $O/lenet_2000.err; exit 1; }
cat $O/lenet_2000.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/lenet_20.json 2>$O/lenet_20.err || exit 1
cat $O/lenet_20.json
ROCKET_BENCH_PROFILE=$O/lenet.prof timeout -k 10 300 python bench.py --steps 3000 --warmup 20 > $O/lenet_prof.json 2>$O/lenet_prof.err || { tail -20 $O/lenet_prof.err; exit 1; }
python - <<'PY' > $O/lenet_host_prof.txt
import pstats
s = pstats.Stats("gpurun_out/r3h/lenet.prof.0")
s.sort_stats("tottime").print_stats(45)
s.sort_stats("cumulative").print_stats(60)
PY
head -120 $O/lenet_host_prof.txt
ROCKET_LENET_TRACE=$O/lenet_step_trace.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/lenet_traced.json 2>$O/lenet_traced.err || { tail -20 $O/lenet_traced.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_step_trace.json'));print(json.dumps(d['spans']))"
