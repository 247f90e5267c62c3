#!/bin/bash
# A/B of the re-tuned bf16 GEMM entries on a second box (alternating, scratch table swaps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T=rocket_amd/tuning/gemm_mi355x.csv
cp $T /tmp/new.csv; cp scripts/archive/r4/tab_prev.csv /tmp/prev.csv
for round in 1 2; do
  for tab in prev new; do
    cp /tmp/$tab.csv $T
    timeout -k 10 200 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4s_$tab.json 2>/dev/null || { cp /tmp/new.csv $T; exit 1; }
    echo "$tab $(python3 -c "import json;r=json.loads(open('gpurun_out/r4s_$tab.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
  done
done
cp /tmp/new.csv $T
