#!/bin/bash
# round 5 box f: BatchNorm folded into the consuming conv (conv.hip BatchNorm-apply prologue) +
# split long-row gather: tests, ResNet-50 / ResNet-18 fold A/B, ResNet-50 kernel trace with the fold
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5f; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_data_ops.py \
  tests/kernels/test_iconv.py tests/kernels/test_norm.py tests/kernels/test_fp16.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in resnet50 resnet18; do
  for v in 1 0 1 0; do
    ROCKET_BN_FOLD=$v timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_$v.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/${m}_$v.json').read().strip().splitlines()[-1]);print('$m fold=$v', r['value'], r['ms_per_step'])"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r50 -o run -- python3 $R/bench.py --model resnet50 --steps 8 --warmup 3 > $O/r50_trace.log 2>&1 || { tail -20 $O/r50_trace.log; exit 1; }
cd $R
f=$(find $O/r50 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ResNet-50 bs256 bf16 step (round 5, BatchNorm folded into the consuming convs), rocprofv3 kernel trace" > gpurun_out/r5_resnet50_fold_kernels.md
rm -rf $O/r50
head -40 gpurun_out/r5_resnet50_fold_kernels.md
