#!/bin/bash
# host-side profile of the fp16 LeNet step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py \
  tests/kernels/test_fp16_vit.py > gpurun_out/r4h_tests.log 2>&1 || { tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -2 gpurun_out/r4h_tests.log
timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4h_vit.json 2>gpurun_out/r4h_vit.err || exit 1
cut -c1-300 gpurun_out/r4h_vit.json
ROCKET_BENCH_PROFILE=gpurun_out/lenet_fp16.prof timeout -k 10 150 python bench.py --mp fp16 --steps 300 --warmup 30 > gpurun_out/r4h_lenet_fp16.json 2>&1 || exit 1
ROCKET_BENCH_PROFILE=gpurun_out/lenet_bf16.prof timeout -k 10 150 python bench.py --steps 300 --warmup 30 > gpurun_out/r4h_lenet_bf16.json 2>&1 || exit 1
python3 - <<'PY'
import pstats
for n in ("fp16", "bf16"):
    print("=====", n)
    pstats.Stats(f"gpurun_out/lenet_{n}.prof.0").sort_stats("tottime").print_stats(22)
PY
