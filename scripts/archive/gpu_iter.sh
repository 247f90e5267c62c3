#!/bin/bash
# quick iteration: kernel tests (no -x), per-kernel timings, fused bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/kernels -m gpu -q > gpurun_out/pytest_kernels.log 2>&1; echo "pytest rc=$?" > gpurun_out/summary.txt
timeout -k 10 300 python bench/lenet_kernels.py > gpurun_out/lenet_kernels.jsonl 2> gpurun_out/lenet_kernels.err; echo "kern rc=$?" >> gpurun_out/summary.txt
timeout -k 10 300 python bench.py --no-graph --steps 100 --warmup 10 > gpurun_out/bench_fused_eager.json 2> gpurun_out/bench_fused_eager.err; echo "bench rc=$?" >> gpurun_out/summary.txt
