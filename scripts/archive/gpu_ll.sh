#!/bin/bash
# Launch-list replay: probe, graph-capture tests, LeNet bench A/B (launch list vs hipGraphLaunch), trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
S=gpurun_out/summary_ll.txt
: > $S
timeout -k 10 120 python bench/graph_launch_probe.py > gpurun_out/graph_probe.json 2> gpurun_out/graph_probe.err; rc=$?; echo "probe rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/gpu/test_graph_capture.py tests/gpu/test_ddp_graph.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ll.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
for i in 1 2; do
  for m in 1 0; do
    ROCKET_LAUNCH_LIST=$m timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/ll_$m_$i.json 2> gpurun_out/ll_$m.err || { echo "bench $m FAILED" >> $S; exit 1; }
    echo "ll=$m $(python -c "import json;d=json.load(open('gpurun_out/ll_$m_$i.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['host_ms_p50'])")" >> $S
  done
done
bash scripts/gpu_prof_lenet.sh
