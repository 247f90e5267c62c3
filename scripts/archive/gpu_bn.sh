#!/bin/bash
# BatchNorm kernels: numerics tests, per-shape fwd+bwd probe, ResNet-50 step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_bn.txt
: > $S
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_norm.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench/bn_probe.py > gpurun_out/bn_probe.jsonl 2> gpurun_out/bn_probe.err; rc=$?; echo "probe rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_resnet50.json 2> gpurun_out/bench_resnet50.err; rc=$?; echo "r50 rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r50 -o run -- python3 $R/bench.py --model resnet50 --steps 5 --warmup 2 > $R/gpurun_out/prof_r50.log 2>&1; rc=$?; echo "prof rc=$rc" >> $R/$S
[ $rc -ne 0 ] && exit 1
cd $R && f=$(find gpurun_out/prof_r50 -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ResNet-50 224^2 bf16 bs256, 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/r50_kernels.md; rc=$?
rm -rf gpurun_out/prof_r50
exit $rc
