#!/bin/bash
# Host-side profile of the LeNet step loop (cProfile over 2000 timed steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/lenet_host.prof bench.py --steps 2000 --warmup 20 > gpurun_out/lenet_host.json 2> gpurun_out/lenet_host.err || exit 1
python - > gpurun_out/lenet_host_prof.txt <<'PY'
import pstats
p = pstats.Stats("gpurun_out/lenet_host.prof")
p.sort_stats("tottime").print_stats(45)
PY
