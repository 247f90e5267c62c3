#!/bin/bash
# mgemm numerics tests, then the ViT-B/16 bench on the native GEMM path
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_mgemm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_mgemm.log 2>&1
rc=$?; tail -5 gpurun_out/test_mgemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/bench_vit.json 2> gpurun_out/bench_vit.err; rc=$?
cat gpurun_out/bench_vit.json; tail -3 gpurun_out/bench_vit.err; exit $rc
