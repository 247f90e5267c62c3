#!/bin/bash
# xgemm5 iteration: numerics (tests + per-tile diag) then the probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6d; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_xgemm5.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench/x5_diag.py > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep -c '"nbad": 0' $O/diag.log
timeout -k 10 300 python bench/gemm_r6_probe.py --out $O/probe.jsonl --shapes ${SHAPES:-qkv,proj,fc1,fc2,qkv_dg,sq8192} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 - <<'PY'
import json,os
for l in open(os.environ.get('GRAFT_REPO_ROOT','.')+'/gpurun_out/r6d/probe.jsonl'):
    r=json.loads(l); print(r['case'], 'lib', r['lib']['tflops'], 'x5', r['x5']['tflops'], r['x5_rel_err'], 'f0', r['f0']['tflops'], 'f1', r['f1']['tflops'], 's1', r['s1']['tflops'], 's8', r['s8']['tflops'], 's9', r['s9']['tflops'], 's10', r['s10']['tflops'])
PY
