#!/bin/bash
# repeat one bench config N times on one box (variance check)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
M=${REP_MODEL:-resnet18}; P=${REP_MP:-fp16}
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model $M --mp $P --steps 40 --warmup 5 > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err || { tail -20 gpurun_out/rep_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rep_$i.json'));print('$M $P',d['value'],d['step_ms_p50'])"
done
