#!/bin/bash
# round 6 box b: persistent GEMM (xgemm5) numerics + probe vs hipBLASLt / xgemm4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6b; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_xgemm5.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python bench/gemm_r6_probe.py --out $O/probe.jsonl > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_mgemm.py -k "x5" > $O/mlin.log 2>&1 || { tail -30 $O/mlin.log; exit 1; }
tail -1 $O/mlin.log
for mode in lib x5; do
  ROCKET_VIT_GEMM=$mode timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$mode.json 2> $O/vit_$mode.err || { tail -20 $O/vit_$mode.err; exit 1; }
  python3 -c "import json;r=json.loads(open('$O/vit_$mode.json').read().strip().splitlines()[-1]);print('vit $mode', r['value'], r['ms_per_step'])"
done
