#!/bin/bash
# LeNet headline: lenet GPU tests, then the driver-shaped bench x3 and a long run
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out; : > gpurun_out/lenet_ab.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "lenet or launch_list or graph_capture" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lenet_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lenet_tests.log >> gpurun_out/lenet_ab.txt; [ $rc -eq 0 ] || { cat gpurun_out/lenet_ab.txt; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', d['value'], d['ms_per_step'], d['step_ms_p50'])" >> gpurun_out/lenet_ab.txt || exit 1
done
timeout -k 10 120 python bench.py 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('long', d['value'], d['ms_per_step'], d['step_ms_p50'])" >> gpurun_out/lenet_ab.txt || exit 1
cat gpurun_out/lenet_ab.txt
