#!/bin/bash
# round 5: same-box A/B (ab_old = HEAD library) of quad-transposed 8-byte dQ/dK/dV stores in the
# fused attention backward: attention tests on the new build, attention probe and ViT-B/16 bf16
# alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5aq; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py tests/kernels/test_fp16_vit.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new old; do
  if [ $v = old ]; then export ROCKET_LIBDIR=$R/ab_old; else unset ROCKET_LIBDIR; fi
  timeout -k 10 120 python bench/attn_probe.py > $O/probe_$v.json 2>> $O/err.log || exit 1
  echo "probe $v $(tail -1 $O/probe_$v.json)"
  timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$v.json 2>> $O/err.log || exit 1
  python3 -c "import json;r=json.loads(open('$O/vit_$v.json').read().strip().splitlines()[-1]);print('vit $v', r['value'], r['ms_per_step'])"
done
