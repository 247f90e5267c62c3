#!/bin/bash
# Full GPU tests, LeNet phase timeline, headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_tl.txt
: > $S
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python bench/lenet_timeline.py > gpurun_out/lenet_timeline.jsonl 2> gpurun_out/lenet_timeline.err; rc=$?; echo "timeline rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?; echo "bench rc=$rc" >> $S
exit $rc
