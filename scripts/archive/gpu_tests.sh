#!/bin/bash
# Full GPU test suite (no -x: every failure is listed), then the driver-shaped bench once.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > gpurun_out/summary.txt
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log >> gpurun_out/summary.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit 1
cat gpurun_out/bench_driver.json >> gpurun_out/summary.txt
