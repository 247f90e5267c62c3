#!/bin/bash
# round 5: 256x256 forward conv tiles (ROCKET_CONV_PIPE 6 = 16 waves, 7 = 8 waves) vs the 128x128
# default: per-shape probe with output check, conv tests on pipeline 6 and 7, ResNet-50 alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5big; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python bench/iconv_probe.py --model resnet50 --cfgs 0,6,7 --check --dirs fwd > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
tail -3 $O/probe.jsonl
for p in 6 7; do
  ROCKET_CONV_PIPE=$p timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_iconv.py > $O/tests_$p.log 2>&1 || { tail -30 $O/tests_$p.log; exit 1; }
  echo "pipe $p: $(tail -1 $O/tests_$p.log)"
done
for pass in 1 2; do
  for p in 0 6 7; do
    ROCKET_CONV_PIPE=$p timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${p}_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/r50_${p}_$pass.json').read().strip().splitlines()[-1]);print('r50 pipe=$p pass=$pass', r['value'], r['ms_per_step'])"
  done
done
