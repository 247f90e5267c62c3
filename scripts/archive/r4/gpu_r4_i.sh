#!/bin/bash
# conv grouped tile walk A/B (ResNet-50 / ResNet-18), conv + mgemm numerics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_iconv.py \
  tests/kernels/test_mgemm.py > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4i_lf16 -o run -- python3 $R/bench.py --mp fp16 --steps 40 --warmup 10 > $R/gpurun_out/r4i_lf16.log 2>&1 || { tail -20 $R/gpurun_out/r4i_lf16.log; exit 1; }
cd $R
f=$(find gpurun_out/r4i_lf16 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 20 --marker mlp3_wgrad --title "LeNet bs1024 fp16 step (round 4), kernel trace" > gpurun_out/r4_lenet_fp16_kernels.md || true
rm -rf gpurun_out/r4i_lf16
head -30 gpurun_out/r4_lenet_fp16_kernels.md
for round in 1 2; do
for g in 1 4; do
  ROCKET_CONV_TILE_GROUP=$g timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r4i_rn50_g$g.json 2>/dev/null || exit 1
  echo "rn50 g=$g $(python3 -c "import json;r=json.load(open('gpurun_out/r4i_rn50_g$g.json'));print(r['value'], r['ms_per_step'])")"
done
done
for g in 1 4; do
  ROCKET_CONV_TILE_GROUP=$g timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r4i_rn18_g$g.json 2>/dev/null || exit 1
  echo "rn18 g=$g $(python3 -c "import json;r=json.load(open('gpurun_out/r4i_rn18_g$g.json'));print(r['value'], r['ms_per_step'])")"
done
