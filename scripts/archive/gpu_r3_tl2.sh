#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3t; export TMPDIR=/tmp
O=$R/gpurun_out/r3t
for ao in 1 0; do
ROCKET_GATHER_ANY_ORDER=$ao ROCKET_LENET_TRACE=$O/trace_ao$ao.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/traced.json 2>$O/traced.err || { tail -20 $O/traced.err; exit 1; }
python -c "import json;d=json.load(open('$O/trace_ao$ao.json'))['spans'];print('any_order=$ao', json.dumps({k:d[k] for k in ('fwd','bwd','wgrad','next_batch_gather')}))"
done
