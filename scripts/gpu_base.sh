#!/bin/bash
# Round-start baseline: GPU suite + smoke + driver-shaped LeNet bench + ViT bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=gpurun_out/base_summary.txt; : > $S
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/base_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $S; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/base_pytest.log >> $S
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/base_lenet.json 2> gpurun_out/base_lenet.err || exit 1
cat gpurun_out/base_lenet.json >> $S
timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/base_vit.json 2> gpurun_out/base_vit.err || exit 1
cat gpurun_out/base_vit.json >> $S
cat $S
