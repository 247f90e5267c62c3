#!/bin/bash
# Host-side cProfile of the LeNet bench loop (per-step Python cost of the capsule tree).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/hp_warm.json 2>&1 || exit 1
timeout -k 10 180 python -m cProfile -o gpurun_out/host.prof bench.py --steps 4000 --warmup 50 > gpurun_out/hp_prof.json 2>&1 || exit 1
python - <<'PY' > gpurun_out/host_prof.txt
import pstats
p = pstats.Stats("gpurun_out/host.prof")
p.sort_stats("cumulative").print_stats(r"rocket_amd|torch/cuda|torch/optim|torch/autograd|torch/_tensor", 70)
p.sort_stats("tottime").print_stats(40)
PY
rm -f gpurun_out/host.prof
timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/hp_bench.json 2>&1 || exit 1
exit 0
