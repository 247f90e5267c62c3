#!/bin/bash
# quick regression: all GPU tests + lenet + vit bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_quick.txt
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/summary_quick.txt
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
timeout -k 10 300 python bench.py --steps 1000 --warmup 20 > gpurun_out/bench_lenet.json 2> gpurun_out/bench_lenet.err; echo "lenet rc=$?" >> gpurun_out/summary_quick.txt
for m in ${MODELS:-vit_b16}; do
timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err; echo "$m rc=$?" >> gpurun_out/summary_quick.txt
done
