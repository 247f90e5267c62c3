#!/bin/bash
# graph-capture check: GPU tests, eager vs graph bench, kernel profile + host profile of graph bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" > gpurun_out/summary.txt
timeout -k 10 300 python bench.py --no-graph --steps 200 --warmup 20 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err; echo "eager rc=$?" >> gpurun_out/summary.txt
timeout -k 10 300 python bench.py --steps 1000 --warmup 20 > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || { echo "graph rc=$?" >> gpurun_out/summary.txt; exit 1; }
echo "graph rc=0" >> gpurun_out/summary.txt
timeout -k 10 300 python -m cProfile -s tottime bench.py --steps 2000 --warmup 20 > gpurun_out/cprofile.txt 2>&1; echo "cprof rc=$?" >> gpurun_out/summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_graph -o run -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/prof_graph.log 2>&1; echo "prof rc=$?" >> gpurun_out/summary.txt
