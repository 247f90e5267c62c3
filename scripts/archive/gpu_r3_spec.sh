#!/bin/bash
# speculative whole-step LeNet launch: tests, bench (driver config + long), captured-step trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3s; export TMPDIR=/tmp
O=$R/gpurun_out/r3s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py tests/kernels/test_ce_optim.py tests/gpu/test_graph_capture.py tests/gpu/test_launcher_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/lenet_20.json 2>$O/lenet_20.err || { tail -20 $O/lenet_20.err; exit 1; }
cat $O/lenet_20.json
timeout -k 10 200 python bench.py --steps 2000 --warmup 20 > $O/lenet_2000.json 2>$O/lenet_2000.err || { tail -20 $O/lenet_2000.err; exit 1; }
cat $O/lenet_2000.json
ROCKET_LENET_SPEC=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 20 > $O/lenet_2000_nospec.json 2>$O/lenet_2000_nospec.err || exit 1
cat $O/lenet_2000_nospec.json
ROCKET_LENET_TRACE=$O/lenet_step_trace.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/lenet_traced.json 2>$O/lenet_traced.err || { tail -20 $O/lenet_traced.err; exit 1; }
python -c "import json;d=json.load(open('$O/lenet_step_trace.json'));print(json.dumps(d['spans']))"
