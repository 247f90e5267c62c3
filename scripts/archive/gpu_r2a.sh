#!/bin/bash
# Round-2 first GPU pass: full GPU test suite, then the driver-shaped LeNet bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" > gpurun_out/summary.txt
tail -3 gpurun_out/pytest_gpu.log >> gpurun_out/summary.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$i.json 2> gpurun_out/bench_driver_$i.err || exit 1
done
timeout -k 10 120 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_*.json >> gpurun_out/summary.txt
