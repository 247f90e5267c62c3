#!/bin/bash
# ViT path: attention/LN kernel tests, ViT-B/16 bench, steady-state kernel trace summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_vit.txt
: > $S
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_vit.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/bench_vit_b16.json 2> gpurun_out/bench_vit_b16.err; rc=$?; echo "vit rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vit.log 2>&1; rc=$?; echo "prof rc=$rc" >> $R/$S
[ $rc -ne 0 ] && exit 1
cd $R && f=$(find gpurun_out/prof_vit -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ViT-B/16 224^2 bf16 bs128, 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/vit_kernels.md; rc=$?
rm -rf gpurun_out/prof_vit
exit $rc
