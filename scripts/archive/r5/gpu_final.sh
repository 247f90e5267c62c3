#!/bin/bash
# Round-5 evidence run: full GPU suite, smoke, driver-shaped + long LeNet bench, model benches
# (bf16; fp16 LeNet / ViT), one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=gpurun_out/final5_summary.txt; : > $S
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/final5_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $S; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/final5_pytest.log >> $S
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final5_smoke.log 2>&1 || exit 1
echo "smoke ok" >> $S
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final5_lenet_driver.json 2> gpurun_out/final5_lenet_driver.err || exit 1
timeout -k 10 120 python bench.py > gpurun_out/final5_lenet_long.json 2> gpurun_out/final5_lenet_long.err || exit 1
timeout -k 10 120 python bench.py --mp fp16 > gpurun_out/final5_lenet_fp16.json 2> gpurun_out/final5_lenet_fp16.err || exit 1
for m in resnet18 resnet50 vit_b16; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/final5_$m.json 2> gpurun_out/final5_$m.err || exit 1
done
timeout -k 10 400 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/final5_vit_b16_fp16.json 2> gpurun_out/final5_vit_b16_fp16.err || exit 1
for f in lenet_driver lenet_long lenet_fp16 resnet18 resnet50 vit_b16 vit_b16_fp16; do
  python3 -c "import json,sys;r=json.loads(open('gpurun_out/final5_$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['dtype'])" >> $S
done
cat $S
for f in gpurun_out/final5_*.json; do tail -1 $f; done > gpurun_out/r5_final_regression.jsonl
