#!/bin/bash
# Round regression on one MI355X: GPU tests, smoke, LeNet bench, optional model benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_round.txt
: > $S
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?; echo "bench rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
for m in ${MODELS:-}; do
timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err; rc=$?; echo "$m rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
done
exit 0
