#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_bn.txt
timeout -k 10 300 python -m pytest tests/kernels/test_norm.py -q -m gpu > gpurun_out/pytest_norm.log 2>&1; echo "pytest rc=$?" >> gpurun_out/summary_bn.txt
timeout -k 10 300 python bench/bn_probe.py > gpurun_out/bn_probe.jsonl 2> gpurun_out/bn_probe.err; echo "probe rc=$?" >> gpurun_out/summary_bn.txt
timeout -k 10 400 python bench.py --model resnet50 --no-graph --steps 20 --warmup 5 > gpurun_out/bench_resnet50_eager.json 2> gpurun_out/bench_resnet50_eager.err; echo "r50 rc=$?" >> gpurun_out/summary_bn.txt
