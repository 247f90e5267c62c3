#!/bin/bash
# round 5: same-box A/B (ab_old = HEAD library) of write-through stores for the LeNet step kernel's
# outputs: LeNet tests on the new build, then driver-shape / long benches alternating + timelines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5wt; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py tests/kernels/test_fp16.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new old; do
  if [ $v = old ]; then export ROCKET_LIBDIR=$R/ab_old; else unset ROCKET_LIBDIR; fi
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$v.json 2>> $O/err.log || exit 1
  timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_$v.json 2>> $O/err.log || exit 1
  for f in drv_$v long_$v; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'])"; done
done
unset ROCKET_LIBDIR
ROCKET_LENET_TRACE=$O/tl_new.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl.json 2>>$O/err.log || exit 1
python3 -c "
import json; d=json.load(open('$O/tl_new.json')); s=d['spans']
print('new', json.dumps({k: s[k] for k in ('fwd','bwd','wgrad')}))"
