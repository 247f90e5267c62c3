#!/bin/bash
# Round-end evidence: full GPU suite, smoke, driver-shaped + long LeNet bench, model benches,
# LeNet kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=gpurun_out/final_summary.txt; : > $S
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/final_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $S; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/final_pytest.log >> $S
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_lenet_driver.json 2> gpurun_out/final_lenet_driver.err || exit 1
timeout -k 10 120 python bench.py > gpurun_out/final_lenet_long.json 2> gpurun_out/final_lenet_long.err || exit 1
for m in resnet18 resnet50 vit_b16; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/final_$m.json 2> gpurun_out/final_$m.err || exit 1
done
bash scripts/gpu_prof_lenet.sh
