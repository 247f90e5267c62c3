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
# variants: "xplain wgradlds" (default: 0 1)
for v in "0 1" "1 1" "0 0" "0 1" "1 1" "0 0"; do
  set -- $v; t="x$1_l$2"
  ROCKET_LENET_X_PLAIN=$1 ROCKET_WGRAD_LDS=$2 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$t.json 2>> $O/err.log || exit 1
  ROCKET_LENET_X_PLAIN=$1 ROCKET_WGRAD_LDS=$2 timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_$t.json 2>> $O/err.log || exit 1
  for f in drv_$t long_$t; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"; done
done
for v in "0 1" "1 1" "0 0"; do
  set -- $v; t="x$1_l$2"
  ROCKET_LENET_X_PLAIN=$1 ROCKET_WGRAD_LDS=$2 ROCKET_LENET_TRACE=$O/timeline_$t.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl_$t.json 2>>$O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/timeline_$t.json')); s=d['spans']; g=d['spans']['wgrad_groups']; print('$t', 'bwd_end', s['bwd']['last_end'], 'wgrad', s['wgrad']['first_start'], s['wgrad']['median_end'], s['wgrad']['last_end'], 'fc1 loop_done', g['fc1 tiles']['median_loop_done'])"
done
O=$R/gpurun_out/r5e; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_xgemm4.py \
  tests/kernels/test_mgemm.py tests/kernels/test_fp16_vit.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  ROCKET_VIT_X4_MLP=$v timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$v.json 2>> $O/err.log || exit 1
  python3 -c "import json;r=json.loads(open('$O/vit_$v.json').read().strip().splitlines()[-1]);print('x4_mlp=$v', r['value'], r['ms_per_step'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/vit -o run -- python3 $R/bench.py --model vit_b16 --steps 8 --warmup 3 > $O/vit_trace.log 2>&1 || { tail -20 $O/vit_trace.log; exit 1; }
cd $R
f=$(find $O/vit -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 bf16 step (round 5, fused x4 MLP GEMMs), rocprofv3 kernel trace" > gpurun_out/r5_vit_b16_kernels.md
rm -rf $O/vit
head -30 gpurun_out/r5_vit_b16_kernels.md
