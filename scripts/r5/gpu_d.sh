#!/bin/bash
# round 5 box d: LeNet KeepSmem part 2 (labels, logits, ReLU masks, dgrad fragments resident) +
# x write-back A/B (non-temporal vs plain): tests, driver bench, long bench, step timelines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5d; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py \
  tests/kernels/test_fp16.py tests/kernels/test_amp.py tests/kernels/test_ce_optim.py tests/kernels/test_data_ops.py \
  tests/gpu/test_graph_capture.py tests/gpu/test_launcher_gpu.py tests/gpu/test_device_loader_gpu.py tests/examples > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1; do
  ROCKET_LENET_X_PLAIN=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$v.json 2>> $O/err.log || exit 1
  ROCKET_LENET_X_PLAIN=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_$v.json 2>> $O/err.log || exit 1
  for f in drv_$v long_$v; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"; done
done
for v in 0 1; do
  ROCKET_LENET_X_PLAIN=$v ROCKET_LENET_TRACE=$O/timeline_$v.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl_$v.json 2>>$O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/timeline_$v.json')); s=d['spans']; print('x_plain=$v', 'bwd_end', s['bwd']['last_end'], 'wgrad', s['wgrad']['first_start'], s['wgrad']['median_end'], s['wgrad']['last_end'])"
done
