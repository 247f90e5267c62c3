#!/bin/bash
# Kernel numerics + smoke + fused-path bench (eager).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/kernels -m gpu -x -q > gpurun_out/pytest_kernels.log 2>&1; echo "pytest rc=$?" > gpurun_out/summary.txt
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?" >> gpurun_out/summary.txt
timeout -k 10 300 python bench.py --no-graph --steps 100 --warmup 10 > gpurun_out/bench_fused_eager.json 2> gpurun_out/bench_fused_eager.err; echo "bench rc=$?" >> gpurun_out/summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fused -- python $R/bench.py --no-graph --steps 30 --warmup 5 > $R/gpurun_out/prof_fused.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/summary.txt
