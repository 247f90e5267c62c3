#!/bin/bash
# Re-tune the bf16 ViT GEMM shapes with a longer TunableOp budget per shape and A/B the result
# against the shipped table (scratch copies on the box; nothing here edits the repo's table)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T=rocket_amd/tuning/gemm_mi355x.csv
cp $T /tmp/orig.csv
grep "^Validator" /tmp/orig.csv > $T
grep "Half" /tmp/orig.csv >> $T
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=400 ROCKET_TUNE_GEMMS=1 ROCKET_TUNED_GEMMS_OUT=$R/gpurun_out/r4p_bf16.csv \
  timeout -k 10 900 python bench.py --model vit_b16 --steps 3 --warmup 2 --no-graph > gpurun_out/r4p_tune.log 2>&1 || { tail -20 gpurun_out/r4p_tune.log; cp /tmp/orig.csv $T; exit 1; }
grep "^Validator" /tmp/orig.csv > /tmp/new.csv
grep "BFloat16" gpurun_out/r4p_bf16.csv >> /tmp/new.csv
grep "Half" /tmp/orig.csv >> /tmp/new.csv
grep -c BFloat16 /tmp/new.csv
for round in 1 2; do
  for tab in orig new; do
    cp /tmp/$tab.csv $T
    timeout -k 10 200 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4p_$tab.json 2>/dev/null || { cp /tmp/orig.csv $T; exit 1; }
    echo "$tab $(python3 -c "import json;r=json.loads(open('gpurun_out/r4p_$tab.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
  done
done
cp /tmp/orig.csv $T
