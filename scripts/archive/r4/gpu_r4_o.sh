#!/bin/bash
# TunableOp table for the fp16 ViT-B/16 GEMM shapes: tune (eager warm-up steps hit every shape),
# merge into a scratch copy of the package table, re-measure fp16 and bf16 ViT with it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4o_vit16_before.json 2>/dev/null || exit 1
ROCKET_TUNE_GEMMS=1 ROCKET_TUNED_GEMMS_OUT=$R/gpurun_out/r4o_tuned_fp16.csv timeout -k 10 600 python bench.py --model vit_b16 --mp fp16 --steps 3 --warmup 2 --no-graph > gpurun_out/r4o_tune.log 2>&1 || { tail -20 gpurun_out/r4o_tune.log; exit 1; }
grep -c "Half" gpurun_out/r4o_tuned_fp16.csv
grep "Half" gpurun_out/r4o_tuned_fp16.csv >> rocket_amd/tuning/gemm_mi355x.csv
timeout -k 10 200 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4o_vit16_after.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4o_vit_bf16.json 2>/dev/null || exit 1
for f in vit16_before vit16_after vit_bf16; do
  echo "$f $(python3 -c "import json;r=json.loads(open('gpurun_out/r4o_$f.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
done
