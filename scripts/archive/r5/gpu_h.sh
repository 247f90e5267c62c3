#!/bin/bash
# round 5 box h/i: LeNet phase C (dW1) with wave-uniform k-steps, conv1 row-tile walk: tests, benches, timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-r5h}; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py \
  tests/kernels/test_fp16.py tests/kernels/test_amp.py tests/gpu/test_graph_capture.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_$i.json 2>> $O/err.log || exit 1
  for f in drv_$i long_$i; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"; done
done
timeout -k 10 120 python bench.py --mp fp16 --steps 1000 --warmup 50 > $O/fp16.json 2>> $O/err.log || exit 1
python3 -c "import json;r=json.loads(open('$O/fp16.json').read().strip().splitlines()[-1]);print('fp16', r['value'], r['ms_per_step'])"
ROCKET_LENET_TRACE=$O/timeline.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl.json 2>>$O/err.log || exit 1
python3 -c "
import json; d=json.load(open('$O/timeline.json')); s=d['spans']
print('fwd end', s['fwd']['median_end'], 'bwd end', s['bwd']['median_end'], s['bwd']['last_end'], 'wgrad', s['wgrad']['first_start'], s['wgrad']['median_end'], s['wgrad']['last_end'])
for k,v in d['waves'].items(): print(k, v)
for p in d['fwd_phases']+d['bwd_phases']: print(p['phase'], p['median_us_since_prev'])"
