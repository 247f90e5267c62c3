#!/bin/bash
# any-order batch gather: loader test + LeNet bench (driver config, long) + step trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3a; export TMPDIR=/tmp
O=$R/gpurun_out/r3a
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_device_loader_gpu.py tests/gpu/test_launcher_gpu.py tests/gpu/test_graph_capture.py tests/gpu/test_models.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/lenet_20_$i.json 2>$O/lenet_20.err || { tail -20 $O/lenet_20.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_20_$i.json'));print('20 steps', d['value'], d['ms_per_step'], d['host_issue_ms'])"
done
timeout -k 10 200 python bench.py --steps 2000 --warmup 20 > $O/lenet_2000.json 2>$O/lenet_2000.err || { tail -20 $O/lenet_2000.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_2000.json'));print('2000 steps', d['value'], d['ms_per_step'], d['host_issue_ms'], d['host_ms_p50'])"
ROCKET_GATHER_ANY_ORDER=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 20 > $O/lenet_2000_ordered.json 2>$O/lenet_2000_o.err || exit 1
python -c "import json;d=json.load(open('$O/lenet_2000_ordered.json'));print('2000 steps ordered gather', d['value'], d['ms_per_step'])"
ROCKET_LENET_TRACE=$O/lenet_step_trace.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/lenet_traced.json 2>$O/lenet_traced.err || { tail -20 $O/lenet_traced.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_step_trace.json'));print(json.dumps(d['spans']))"
