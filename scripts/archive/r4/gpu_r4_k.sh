#!/bin/bash
# host-side cProfile of the fp16 / bf16 LeNet steps (bench.py ROCKET_BENCH_PROFILE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
ROCKET_BENCH_PROFILE=gpurun_out/k_lenet_fp16.prof timeout -k 10 200 python bench.py --mp fp16 > gpurun_out/k_lenet_fp16.json 2>&1 || exit 1
ROCKET_BENCH_PROFILE=gpurun_out/k_lenet_bf16.prof timeout -k 10 200 python bench.py > gpurun_out/k_lenet_bf16.json 2>&1 || exit 1
tail -c 600 gpurun_out/k_lenet_fp16.json
