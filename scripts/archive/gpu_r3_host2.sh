#!/bin/bash
# LeNet host-side cost per step: cProfile of a long run (tottime / cumulative tables)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3h; export TMPDIR=/tmp
O=$R/gpurun_out/r3h
ROCKET_BENCH_PROFILE=$O/lenet.prof timeout -k 10 300 python bench.py --steps 3000 --warmup 20 > $O/lenet_prof.json 2>$O/lenet_prof.err || { tail -20 $O/lenet_prof.err; exit 1; }
python - <<'PY' > $O/lenet_host_prof.txt
import pstats
s = pstats.Stats("gpurun_out/r3h/lenet.prof.0")
s.sort_stats("tottime").print_stats(50)
s.sort_stats("cumulative").print_stats(70)
PY
