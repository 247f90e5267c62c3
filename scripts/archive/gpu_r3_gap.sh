#!/bin/bash
# kernel-boundary gap vs bytes written; LeNet captured-step trace with wgrad block groups
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3g; export TMPDIR=/tmp
O=$R/gpurun_out/r3g
timeout -k 10 120 python bench/gap_probe.py > $O/gap.jsonl 2>$O/gap.err || { tail -20 $O/gap.err; exit 1; }
cat $O/gap.jsonl
ROCKET_LENET_TRACE=$O/lenet_step_trace.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/lenet_traced.json 2>$O/lenet_traced.err || { tail -20 $O/lenet_traced.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_step_trace.json'));print(json.dumps(d['spans']))"
