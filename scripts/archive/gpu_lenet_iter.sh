#!/bin/bash
# LeNet kernel iteration: kernel + graph tests, phase timeline, 3 bench runs (1000 steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_iter.txt
: > $S
timeout -k 10 600 python -u -m pytest tests/kernels tests/gpu/test_graph_capture.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python bench/lenet_timeline.py > gpurun_out/lenet_timeline.jsonl 2> gpurun_out/lenet_timeline.err; rc=$?; echo "timeline rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/iter_$i.json 2> gpurun_out/iter_$i.err || { echo "bench FAILED" >> $S; exit 1; }
  echo "bench $(python -c "import json;d=json.load(open('gpurun_out/iter_$i.json'));print(d['value'],d['ms_per_step'],d['host_ms_p50'])")" >> $S
done
exit 0
