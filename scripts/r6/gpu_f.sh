#!/bin/bash
# xgemm5 numerics + ViT-B/16 in-model A/B (lib vs x5), then the GEMM probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6f; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_xgemm5.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_mgemm.py -k "x5" > $O/mlin.log 2>&1 || { tail -30 $O/mlin.log; exit 1; }
tail -1 $O/mlin.log
for mode in ${MODES:-lib x5}; do
  ROCKET_VIT_GEMM=$mode timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$mode.json 2> $O/vit_$mode.err || { tail -20 $O/vit_$mode.err; exit 1; }
  python3 -c "import json;r=json.loads(open('$O/vit_$mode.json').read().strip().splitlines()[-1]);print('vit $mode', r['value'], r['ms_per_step'])"
done
timeout -k 10 300 python bench/gemm_r6_probe.py --out $O/probe.jsonl --rounds 2 --shapes ${SHAPES:-qkv,proj,fc1,fc2,qkv_dg,fc1_dg} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 - <<'PY'
import json,os
for l in open(os.environ.get('GRAFT_REPO_ROOT','.')+'/gpurun_out/r6f/probe.jsonl'):
    r=json.loads(l); print(r['case'], 'lib', r['lib']['tflops'], 'x5', r['x5']['tflops'], r['x5_rel_err'])
PY
