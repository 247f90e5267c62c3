#!/bin/bash
# Round 3 batch e: fp16 native kernels (tests + ResNet-18 fp16 kernel trace), bf16 regressions,
# ResNet bench numbers with the host issue time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3e; export TMPDIR=/tmp
O=$R/gpurun_out/r3e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_fp16.py tests/kernels/test_iconv.py tests/kernels/test_norm.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/$m.json 2>$O/$m.err || { tail -20 $O/$m.err; exit 1; }
  echo "$m bf16: $(cat $O/$m.json)"
done
timeout -k 10 300 python bench.py --model resnet18 --mp fp16 --steps 20 --warmup 5 > $O/resnet18_fp16.json 2>$O/resnet18_fp16.err || { tail -20 $O/resnet18_fp16.err; exit 1; }
echo "resnet18 fp16: $(cat $O/resnet18_fp16.json)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr16 -o run -- python3 $R/bench.py --model resnet18 --mp fp16 --steps 6 --warmup 3 > $O/tr16.log 2>&1 || { tail -20 $O/tr16.log; exit 1; }
f=$(find $O/tr16 -name '*kernel_trace.csv' | head -1)
cd $R && python3 bench/summarize_trace.py "$f" --steps 4 --title "ResNet-18 (CIFAR) bs256 fp16, 1x MI355X - rocprofv3 --kernel-trace (round 3)" > $O/resnet18_fp16_kernels.md && rm -rf $O/tr16
head -30 $O/resnet18_fp16_kernels.md
